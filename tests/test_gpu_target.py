"""PMML ``Target`` post-processing on the device epilogue (csrc/epilogue.h ``apply_target``):
clip to [min, max], rescale, castInteger, TargetValue defaultValue — tree ensembles, a GLM with a
link function followed by a rescale, the fused MLP and the GEMM MLP — vs the float64 oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cmp(gpu, txt, F=None, missing=0.0, n=20_000, tol=1e-4, X=None, **kw):
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **kw)
    if X is None:
        X = stream_matrix(n, F or c.n_features, seed=3, missing_rate=missing)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    close = np.abs(s[v] - ref[v]) <= tol
    return plan, close.mean(), s, ref


@pytest.mark.parametrize("cast", [None, "round", "ceiling", "floor"])
def test_tree_target_clip_rescale_cast(gpu, cast):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, set_target

    txt = set_target(gbdt_pmml(n_trees=50, depth=5, n_features=8, seed=2), min=-0.2, max=0.25, factor=10.0,
                     constant=3.0, cast=cast)
    plan, agree, s, _ = _cmp(gpu, txt, 8, missing=0.02)
    assert "tgt" in plan.epi_args
    # castInteger: only values within fp32 noise of a rounding boundary may differ
    assert agree > (0.999 if cast else 0.99999)
    v = ~np.isnan(s)
    # clip [-0.2, 0.25] * 10 + 3 (fp64: -0.2 * 10 + 3 = 0.9999999999999996, which floors to 0)
    assert s[v].min() >= (0.0 if cast == "floor" else 1.0) - 1e-5 and s[v].max() <= 6.0 + 1e-5


def test_tree_target_default_value(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, set_target

    txt = set_target(gbdt_pmml(n_trees=20, depth=4, n_features=6, seed=1, missing_strategy="nullPrediction"),
                     default=-5.0)
    plan, agree, s, ref = _cmp(gpu, txt, 6, missing=0.1)
    assert agree == 1.0 and (s == -5.0).any() and (s != -5.0).any()


def test_glm_link_then_rescale(gpu):
    from flink_jpmml_amd.bench.synth import glm_pmml, set_target

    from flink_jpmml_amd.bench.synth import mixed_records

    txt = set_target(glm_pmml(model_type="generalizedLinear", link="log", n_features=3, seed=1), max=3.0,
                     factor=0.5, constant=1.0)
    _, X = mixed_records(20_000, 3, seed=2)  # valid vocabulary codes in the categorical column
    plan, agree, s, _ = _cmp(gpu, txt, X=X, tol=1e-4)
    assert agree > 0.9999 and np.nanmax(s) <= 2.5 + 1e-6


@pytest.mark.parametrize("kind", ["fused", "gemm"])
def test_mlp_target(gpu, kind):
    from flink_jpmml_amd.bench.synth import mlp_pmml, set_target

    txt = set_target(mlp_pmml(n_features=8, hidden=(32, 16), n_out=1, seed=4), min=-0.5, max=0.5, factor=10.0,
                     cast="floor")
    opts = {} if kind == "fused" else {"mlp_impl": "gemm"}
    plan, agree, _, _ = _cmp(gpu, txt, 8, **opts)
    assert plan.kind == ("mlp" if kind == "fused" else "mlp_gemm")
    assert agree > 0.999


@pytest.mark.parametrize("impl", ["fused", "wide", "gemm"])
@pytest.mark.parametrize("kw", [dict(min=-0.5, max=0.5, factor=10.0, cast="floor"),
                                dict(factor=3.0, constant=-1.0),
                                dict(default=7.0, cast="round")], ids=["clip-cast", "rescale", "default"])
def test_svm_regression_target(gpu, impl, kw):
    """A regression SVM's Target (clip, rescale, castInteger, TargetValue defaultValue for rows
    without a prediction) on all three SVM plans — the kernels used to write the raw decision
    value (the oracle applies the Target to every regression model)."""
    from flink_jpmml_amd.bench.synth import set_target, svm_pmml

    txt = set_target(svm_pmml(n_features=12, n_sv=64, seed=5, classification=False), **kw)
    plan, agree, s, ref = _cmp(gpu, txt, 12, missing=0.05, svm_impl=impl)
    assert agree > 0.999
