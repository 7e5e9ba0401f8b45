"""Segmented MiningModels (selectFirst / max / median / predicates / non-tree segments) on the GPU:
real segment kernels + device predicates + tensor aggregation vs the float64 oracle. CPU twin:
tests/test_segmented.py."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(gpu, txt, n=20_000, missing=0.05):
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = stream_matrix(n, c.n_features, seed=4, missing_rate=missing)
    s, v = plan.score(X)
    ref, vref = c.score_matrix_oracle(X)
    return plan, s.cpu().numpy(), v.cpu().numpy(), ref, vref


@pytest.mark.parametrize("method", ["selectFirst", "max", "median", "weightedAverage", "weightedMedian"])
def test_regression_segmentation_on_gpu(gpu, method):
    from flink_jpmml_amd.bench.synth import segmented_pmml

    plan, s, v, ref, vref = _run(gpu, segmented_pmml(method, False, n_segments=5, seed=7))
    assert type(plan).__name__ in ("SegmentedPlan", "DerivedPlan")
    assert (v == vref).all() and v.any()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("method", ["majorityVote", "selectFirst", "average", "weightedAverage", "max", "median"])
def test_classification_segmentation_on_gpu(gpu, method):
    from flink_jpmml_amd.bench.synth import segmented_pmml

    plan, s, v, ref, vref = _run(gpu, segmented_pmml(method, True, n_segments=6, n_classes=4, seed=11))
    assert (v == vref).all() and (s[v] == ref[v]).all()


def test_linear_segment_median_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import segmented_pmml

    plan, s, v, ref, vref = _run(gpu, segmented_pmml("median", False, n_segments=4, seed=5, predicates=False,
                                                     linear_segment=True), missing=0.0)
    assert (v == vref).all() and v.all()
    np.testing.assert_allclose(s, ref, rtol=1e-5, atol=1e-5)
