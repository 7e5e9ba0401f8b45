"""Round-3 JPMML surface on the device through the public API with ``fallback="error"`` (a model
that does not lower raises instead of silently taking the host oracle): k-NN with k > 1, ordinal
GLMs, classification average / max / median under segment predicates, regression weightedMedian,
and ``x-mathContext="float"`` ensembles. Each is checked against the host oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bound(gpu, txt):
    from flink_jpmml_amd.api.pmml_model import PmmlModel
    from flink_jpmml_amd.config import ScoringConfig

    m = PmmlModel.from_string(txt).bind(gpu, ScoringConfig(device=gpu, fallback="error"))
    assert m.on_device
    return m


def _check(gpu, txt, X, exact_frac=None, rtol=1e-4, atol=1e-5):
    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    m = _bound(gpu, txt)
    pb = m.predict(RecordBatch(X))
    s, v = pb.scores, pb.valid
    ref, vref = CompiledPmml.from_string(txt).score_matrix_oracle(X)
    assert (v == vref).mean() > 0.999
    both = v & vref
    assert both.any()
    if exact_frac is not None:
        assert (s[both] == ref[both]).mean() >= exact_frac
    else:
        assert np.isclose(s[both], ref[both], rtol=rtol, atol=atol).mean() > 0.998


@pytest.mark.parametrize("k,cls,method", [(5, True, "weightedMajorityVote"), (9, False, "median"),
                                          (16, False, "weightedAverage")])
def test_knn_k_gt_1(gpu, k, cls, method):
    from flink_jpmml_amd.bench.synth import knn_pmml, stream_matrix

    txt = knn_pmml(n_instances=600, n_features=8, k=k, classification=cls, method=method, seed=k)
    _check(gpu, txt, stream_matrix(30_000, 8, seed=1, missing_rate=0.02), exact_frac=0.998 if cls else None)


@pytest.mark.parametrize("link", ["logit", "probit", "cloglog", "cauchit"])
def test_ordinal_glm(gpu, link):
    from flink_jpmml_amd.bench.synth import glm_pmml, mixed_records

    txt = glm_pmml(model_type="ordinalMultinomial", link=link, classes=4, seed=3)
    _, X = mixed_records(30_000, 3, seed=2, missing_rate=0.03)
    _check(gpu, txt, X, exact_frac=0.999)


@pytest.mark.parametrize("method", ["average", "weightedAverage", "max", "median"])
def test_classification_probability_segmentations(gpu, method):
    from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix

    txt = segmented_pmml(method, True, n_segments=6, n_classes=4, seed=11)
    _check(gpu, txt, stream_matrix(30_000, 6, seed=3, missing_rate=0.05), exact_frac=0.999)


def test_weighted_median_segmentation(gpu):
    from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix

    txt = segmented_pmml("weightedMedian", False, n_segments=5, seed=7)
    _check(gpu, txt, stream_matrix(30_000, 6, seed=4, missing_rate=0.05))


def test_float_math_context_ensemble(gpu):
    from test_math_context import _decimal_thresholds, _edge_inputs, _float_ctx

    from flink_jpmml_amd.bench.synth import gbdt_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    txt = _float_ctx(_decimal_thresholds(gbdt_pmml(n_trees=100, depth=6, n_features=10, seed=5)))
    X = _edge_inputs(CompiledPmml.from_string(txt), n=20_000, seed=6)
    _check(gpu, txt, X, rtol=0, atol=2e-6)
