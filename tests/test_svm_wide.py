"""Wide SVMs (one-against-one over many classes, > 64 vector fields) on ``svm_wide_kernel``:
the host packing (support vectors, squared norms and dual coefficients swizzled into the MFMA
fragment order of the two chained products) is checked on the CPU by a numpy emulation of the
kernel's exact operand maps against the float64 oracle; tests/test_gpu_svm_lr.py runs the kernel."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.nn_plans import SvmGemmPlan, SvmWidePlan, _pperm
from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run


def _plan(c, **kw):
    with lowering_dry_run():
        return compile_plan(c, torch.device("cpu"), **kw)


def emulate(plan, X):
    """The kernel's arithmetic on the packed tensors: per 32-vector tile t, G[m][n] = sum over MFMA
    steps q and k in {0, 1} of svA[t, 32k + m, q] * x[n, 2q + k]; register i of lane half h holds
    G[p(i, h)]; the kernel function runs on it; D[32 mt + mm][n] += sum over steps j, k of
    coefA[t, mt, 32k + mm, j] * K[(j, k)][n]. Returns (decision [n, M], bad rows)."""
    Xf = X.astype(np.float32)
    n = len(X)
    idx = plan.in_index.numpy()
    F = plan.n_in
    Q = plan.fmax // 2
    xb = np.zeros((n, plan.fmax), np.float64)
    xb[:, :F] = Xf[:, idx]
    bad = np.isnan(xb).any(1)
    xb = np.nan_to_num(xb)
    xx = (xb ** 2).sum(1)
    svA = plan.svA.numpy().astype(np.float64)      # [T, 64, Q]
    coefA = plan.coefA.numpy().astype(np.float64)  # [T, MT, 64, 16]
    svnP = plan.svnP.numpy().astype(np.float64)    # [T, 2, 16]
    T, MTt = coefA.shape[0], coefA.shape[1]
    D = np.zeros((n, MTt * 32))
    for t in range(T):
        G = np.zeros((n, 32))
        for q in range(Q):
            for k in range(2):
                G += xb[:, 2 * q + k][:, None] * svA[t, 32 * k: 32 * k + 32, q][None, :]
        Kr = np.zeros((n, 2, 16))  # register (h, i)
        for h in range(2):
            for i in range(16):
                g = G[:, _pperm(i, h)]
                kc = plan.kernel_code
                if kc == 2:
                    Kr[:, h, i] = np.exp(-plan.gamma * np.maximum(xx - 2 * g + svnP[t, h, i], 0))
                elif kc == 1:
                    Kr[:, h, i] = (plan.gamma * g + plan.coef0) ** plan.degree
                elif kc == 3:
                    Kr[:, h, i] = np.tanh(plan.gamma * g + plan.coef0)
                else:
                    Kr[:, h, i] = g
        for mt in range(MTt):
            for j in range(16):
                for k in range(2):
                    D[:, 32 * mt: 32 * mt + 32] += coefA[t, mt, 32 * k: 32 * k + 32, j][None, :] * Kr[:, k, j][:, None]
    M = plan.n_machines
    return D[:, :M] + plan.intercept.numpy()[:M][None, :], bad


def finish(plan, D, bad):
    if not plan.classification:
        s = D[:, 0]
    else:
        thr, tgt, alt = plan.thr.numpy(), plan.tgt.numpy(), plan.alt.numpy()
        votes = np.zeros((len(D), plan.n_classes), np.int64)
        for m in range(plan.n_machines):
            first = D[:, m] < thr[m]
            if plan.max_wins:
                first = ~first
            c = np.where(first, tgt[m], alt[m])
            ok = c >= 0
            np.add.at(votes, (np.nonzero(ok)[0], c[ok]), 1)
        s = plan.table.numpy()[votes.argmax(1)]
    return np.where(bad, np.nan, s), ~bad


@pytest.mark.parametrize("kernel", ["radialBasis", "linear", "polynomial", "sigmoid"])
@pytest.mark.parametrize("n_classes,n_feat", [(5, 10), (12, 20), (20, 8)])
def test_wide_svm_packing_matches_oracle(kernel, n_classes, n_feat):
    c = CompiledPmml.from_string(svm_pmml(n_features=n_feat, n_sv=70, seed=4, kernel=kernel, n_classes=n_classes,
                                          gamma=0.1))
    plan = _plan(c)
    assert isinstance(plan, SvmWidePlan)
    M = n_classes * (n_classes - 1) // 2
    assert plan.n_machines == M and plan.mt == (1 if M <= 32 else 2 if M <= 64 else 4)
    assert plan.n_groups == -(-M // (32 * plan.mt))  # 20 classes: 190 machines in 2 groups of 128
    X = stream_matrix(600, n_feat, seed=2, missing_rate=0.01)
    D, bad = emulate(plan, X)
    s, v = finish(plan, D, bad)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.995  # fp32-rounded operands: near-threshold decisions may flip


def test_wide_regression_svm_many_fields():
    c = CompiledPmml.from_string(svm_pmml(n_features=100, n_sv=45, seed=1, classification=False))
    plan = _plan(c)
    assert isinstance(plan, SvmWidePlan) and plan.fmax == 128 and plan.n_tiles == 2
    X = stream_matrix(400, 100, seed=3)
    D, bad = emulate(plan, X)
    s, v = finish(plan, D, bad)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s, ref, rtol=1e-5, atol=1e-5)


def test_wide_svm_routing():
    small = CompiledPmml.from_string(svm_pmml(n_features=8, n_sv=40, seed=2, n_classes=3))
    assert type(_plan(small)).__name__ == "SvmPlan"  # <= 8 machines, <= 64 fields: the fused kernel
    assert isinstance(_plan(small, svm_impl="wide"), SvmWidePlan)
    assert isinstance(_plan(small, svm_impl="gemm"), SvmGemmPlan)
    huge = CompiledPmml.from_string(svm_pmml(n_features=140, n_sv=33, seed=2, classification=False))
    assert isinstance(_plan(huge), SvmGemmPlan)  # > 128 fields: library GEMMs
    with pytest.raises(ValueError):
        _plan(small, svm_impl="nope")


def test_wide_svm_hundreds_of_classes():
    """100 classes = 4950 one-against-one machines in 39 groups of 128: the packed u16 vote
    counters cover up to 256 classes (128 KiB of LDS per 256-row tile); 257 classes go to the
    library-GEMM plan."""
    c = CompiledPmml.from_string(svm_pmml(n_features=6, n_sv=40, seed=3, n_classes=100, gamma=0.3))
    plan = _plan(c)
    assert isinstance(plan, SvmWidePlan) and plan.n_classes == 100
    assert plan.n_machines == 4950 and plan.mt == 4 and plan.n_groups == 39
    X = stream_matrix(150, 6, seed=7, missing_rate=0.01)
    D, bad = emulate(plan, X)
    s, v = finish(plan, D, bad)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.99
    over = CompiledPmml.from_string(svm_pmml(n_features=4, n_sv=8, seed=3, n_classes=SvmWidePlan.CMAX + 1))
    assert isinstance(_plan(over), SvmGemmPlan)
