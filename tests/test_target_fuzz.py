"""Randomized PMML ``Target`` post-processing on the device: a random rescaleFactor /
rescaleConstant, optional min / max clip, castInteger (round / ceiling / floor) and TargetValue
defaultValue on random regression models of every device family (GBDT, single tree with
nullPrediction leaves, RegressionModel with a link, GLM, MLP, SVM, k-NN, segmented selectFirst /
average) — device vs the float64 oracle. The order (rescale → clip → cast; default for rows
without a prediction) is the oracle's; castInteger makes the check exact except at .5 ties of
the fp32 value."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _model(kind: str, seed: int):
    from flink_jpmml_amd.bench import synth

    if kind == "gbdt":
        return synth.gbdt_pmml(n_trees=16, depth=4, n_features=6, seed=seed), 6
    if kind == "regression":
        return synth.regression_design_pmml(n_features=4, normalization="logit", seed=seed), None
    if kind == "glm":
        return synth.glm_pmml(link="log", seed=seed), None
    if kind == "mlp":
        return synth.mlp_pmml(n_features=6, hidden=(12,), seed=seed), 6
    if kind == "svm":
        return synth.svm_pmml(n_features=6, n_sv=30, seed=seed, classification=False), 6
    if kind == "knn":
        return synth.knn_pmml(n_instances=80, n_features=4, k=3, classification=False, seed=seed), 4
    return synth.segmented_pmml(method="average", classification=False, n_segments=5, depth=3, n_features=6,
                                seed=seed, predicates=True), 6


KINDS = ["gbdt", "regression", "glm", "mlp", "svm", "knn", "segmented"]


def _case(seed: int):
    from flink_jpmml_amd.bench.synth import set_target

    rng = np.random.default_rng(3300 + seed)
    kind = KINDS[seed % len(KINDS)]
    txt, F = _model(kind, seed)
    kw = dict(factor=float(rng.choice([1.0, 2.5, -0.75, 100.0])), constant=float(rng.choice([0.0, 0.5, -3.0])))
    if rng.random() < 0.5:
        kw["min"] = float(rng.uniform(-2, 0))
    if rng.random() < 0.5:
        kw["max"] = float(rng.uniform(0.1, 3))
    if rng.random() < 0.4:
        kw["cast"] = str(rng.choice(["round", "ceiling", "floor"]))
    if rng.random() < 0.3:
        kw["default"] = float(rng.choice([-7.0, 42.0]))
    if "min" in kw and "max" in kw and kw["min"] > kw["max"]:
        kw["min"], kw["max"] = kw["max"], kw["min"]
    return kind, set_target(txt, **kw), F, kw


def _inputs(c, F, n, seed):
    from flink_jpmml_amd.bench.synth import mixed_records, stream_matrix

    if F is None:
        return mixed_records(n, len(c.active_fields) - 1, seed=seed, missing_rate=0.03)[1]
    return stream_matrix(n, F, seed=seed, missing_rate=0.03)


@pytest.mark.parametrize("seed", range(14))
def test_random_targets_lower(seed):
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    _, txt, _, _ = _case(seed)
    with lowering_dry_run():
        CompiledPmml.from_string(txt).plan("cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(42, 12))
def test_random_targets_on_gpu(gpu, seed):
    kind, txt, F, kw = _case(seed)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = _inputs(c, F, 5000, seed)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), (seed, kind, kw, int((v != vref).sum()))
    if not v.any():
        return
    scale = max(1.0, float(np.abs(ref[v]).max()))
    diff = np.abs(s[v] - ref[v])
    if "cast" in kw:  # an fp32 value on the other side of an integer / .5 boundary moves by one
        assert (diff > 0).mean() <= 0.01, (seed, kind, kw)
        assert (diff <= 1.0 + 2e-4 * scale).all(), (seed, kind, kw, float(diff.max()))
    else:
        assert (diff <= 2e-4 * scale).all(), (seed, kind, kw, float(diff.max()))
