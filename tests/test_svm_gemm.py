"""The library-GEMM SVM plan (:class:`SvmGemmPlan`: two fp32 GEMMs + element-wise kernel + vote
product) — the fallback beyond the wide MFMA kernel's limits (> 128 vector fields or > 64
classes), and ``svm_impl="gemm"`` on request. Its tensor program runs on the host in a lowering dry run and must match the
float64 oracle (tests/test_gpu_kernels.py runs it on the MI355X)."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.nn_plans import SvmGemmPlan
from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run


def _score(c, X, **kw):
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"), **kw)
        s, v = plan.score(X)
    return plan, s.numpy(), v.numpy().astype(bool)


@pytest.mark.parametrize("kernel", ["radialBasis", "linear", "polynomial", "sigmoid"])
def test_one_against_one_many_classes(kernel):
    c = CompiledPmml.from_string(svm_pmml(n_features=10, n_sv=150, seed=4, kernel=kernel, n_classes=5))
    assert len(c.evaluator.sm.machines) == 10  # > 8: beyond the fused kernel
    X = stream_matrix(3000, 10, seed=2, missing_rate=0.01)
    plan, s, v = _score(c, X, svm_impl="gemm")
    assert isinstance(plan, SvmGemmPlan)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.999  # fp32 decision values near a threshold may flip


def test_wide_regression_svm_and_forced_gemm():
    c = CompiledPmml.from_string(svm_pmml(n_features=80, n_sv=64, seed=1, classification=False))
    X = stream_matrix(2000, 80, seed=3)
    plan, s, v = _score(c, X, svm_impl="gemm")
    assert isinstance(plan, SvmGemmPlan)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s, ref, rtol=1e-4, atol=1e-4)
    c2 = CompiledPmml.from_string(svm_pmml(n_features=8, n_sv=32, seed=2))
    plan2, s2, v2 = _score(c2, stream_matrix(500, 8, seed=1), svm_impl="gemm")
    assert isinstance(plan2, SvmGemmPlan)
