"""Iris multinomial logistic regression probabilities and class index on the linear kernel, and
one-against-one SVMs on the fused kernel (<= 8 machines) and the GEMM path (more machines),
against the float64 oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_iris_logistic_probs_and_argmax(gpu):
    import torch

    from flink_jpmml_amd.bench.synth import iris_logistic_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import LinearPlan

    c = CompiledPmml.from_string(iris_logistic_pmml())
    plan = c.plan(gpu)
    assert isinstance(plan, LinearPlan)
    plan.table = None  # emit the class index instead of the (string) label's numeric value
    plan.__dict__.pop("_args", None)
    rng = np.random.default_rng(0)
    X = rng.uniform([4, 2, 1, 0], [8, 4.5, 7, 2.5], (20_000, 4))
    Xt = torch.from_numpy(X.astype(np.float32)).to(gpu)
    s = torch.empty(len(X), device=gpu)
    v = torch.empty(len(X), dtype=torch.uint8, device=gpu)
    probs = torch.empty((len(X), 3), device=gpu)
    plan.launch(Xt, s, v, probs=probs)
    torch.cuda.synchronize()
    res, _ = c.evaluate_prepared(c.prepare(X.astype(np.float32))[0])
    assert v.cpu().numpy().astype(bool).all()
    np.testing.assert_allclose(probs.cpu().numpy(), res.probs, atol=2e-5)
    lab = s.cpu().numpy()
    agree = (lab == np.argmax(res.probs, axis=1)).mean()
    assert agree > 0.9999  # fp32 vs fp64 near-ties only


@pytest.mark.parametrize("n_classes,kind", [(3, "SvmPlan"), (5, "SvmWidePlan"), (20, "SvmWidePlan")])
def test_one_against_one_svm_on_gpu(gpu, n_classes, kind):
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(svm_pmml(n_features=12, n_sv=160, seed=6, n_classes=n_classes, gamma=0.2))
    plan = c.plan(gpu)
    assert type(plan).__name__ == kind
    X = stream_matrix(30_000, 12, seed=3, missing_rate=0.01)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.999


@pytest.mark.parametrize("kernel", ["radialBasis", "linear", "polynomial", "sigmoid"])
@pytest.mark.parametrize("n_classes,n_feat,n_rows", [(7, 24, 40_000), (12, 70, 20_000), (24, 16, 777)])
def test_wide_svm_kernel_on_gpu(gpu, kernel, n_classes, n_feat, n_rows):
    """svm_wide_kernel (two chained exact-fp32 MFMA products, LDS votes) against the fp64 oracle
    and the library-GEMM plan: 21 / 66 / 276 machines (1 group of 1 tile, 1 group of 4 tiles,
    3 groups of 4 tiles), 24 / 70 / 16 fields, a ragged last tile."""
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(svm_pmml(n_features=n_feat, n_sv=150, seed=8, kernel=kernel, n_classes=n_classes,
                                          gamma=0.08))
    plan = c.plan(gpu)
    assert type(plan).__name__ == "SvmWidePlan"
    X = stream_matrix(n_rows, n_feat, seed=5, missing_rate=0.01)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.998
    g = c.plan(gpu, svm_impl="gemm")
    sg, vg = g.score(X)
    sg = sg.cpu().numpy()
    assert (s[v] == sg[v]).mean() > 0.998


def test_wide_regression_svm_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(svm_pmml(n_features=100, n_sv=300, seed=1, classification=False, gamma=0.01))
    plan = c.plan(gpu)
    assert type(plan).__name__ == "SvmWidePlan" and plan.fmax == 128
    X = stream_matrix(50_000, 100, seed=3, missing_rate=0.005)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n_classes,n_rows", [(100, 5_000), (256, 600)])
def test_wide_svm_hundreds_of_classes_on_gpu(gpu, n_classes, n_rows):
    """4950 / 32640 one-against-one machines (39 / 255 groups of 128) voting into packed u16
    counters of up to 128 KiB of LDS, against the fp64 oracle and the library-GEMM plan."""
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(svm_pmml(n_features=10, n_sv=64, seed=9, n_classes=n_classes, gamma=0.3))
    plan = c.plan(gpu)
    assert type(plan).__name__ == "SvmWidePlan" and plan.n_classes == n_classes
    X = stream_matrix(n_rows, 10, seed=4, missing_rate=0.01)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.99
    sg, _ = c.plan(gpu, svm_impl="gemm").score(X)
    assert (s[v] == sg.cpu().numpy()[v]).mean() > 0.99
