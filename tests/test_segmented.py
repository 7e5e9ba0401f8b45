"""Segmentations the fused ensemble kernels refuse (selectFirst / max / min / median, non-True
segment predicates, non-tree segments) lower to :class:`SegmentedPlan`: per-segment device plans,
device predicates, tensor-op aggregation. CPU check: the plan built in a lowering dry run, with
stand-in segment plans that write the oracle's per-segment results, must reproduce the oracle's
aggregate — this pins the predicate programs and every aggregation rule without a GPU (the GPU
twin, tests/test_gpu_segmented.py, runs the real segment kernels)."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run
from flink_jpmml_amd.runtime.segmented import SegmentedPlan, segmentable


class _OracleSegment:
    """Stand-in segment plan: the oracle's result of one segment model (class index for
    classification, like the real plans with their label table switched off)."""

    def __init__(self, compiled, sub):
        self.c, self.sub = compiled, sub

    def launch(self, X, score, valid, stream=None, **kw):
        cols = self.c.columns(X.double().numpy())
        r = self.sub.evaluate(cols)
        score.copy_(torch.from_numpy(np.where(r.valid, r.value, np.nan)).float())
        valid.copy_(torch.from_numpy(r.valid.astype(np.uint8)))
        if kw.get("probs") is not None:
            kw["probs"].copy_(torch.from_numpy(r.probs).float())


def _run(txt, n=4000, missing=0.08, seed=3):
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, SegmentedPlan)
    plan.subs = [_OracleSegment(c, sub) for sub in c.evaluator.sub]
    X = stream_matrix(n, c.n_features, seed=seed, missing_rate=missing)
    s = torch.empty(n)
    v = torch.empty(n, dtype=torch.uint8)
    plan.launch(torch.from_numpy(X.astype(np.float32)), s, v)
    ref, vref = c.score_matrix_oracle(X.astype(np.float32))
    return plan, s.numpy(), v.numpy().astype(bool), ref, vref


@pytest.mark.parametrize("method", ["selectFirst", "max", "min", "median", "sum", "average", "weightedAverage",
                                    "weightedMedian"])
@pytest.mark.parametrize("treatment", [None, "skipSegment"])
def test_regression_segmentations(method, treatment):
    plan, s, v, ref, vref = _run(segmented_pmml(method, False, n_segments=5, seed=7, missing_treatment=treatment))
    assert (v == vref).all()
    assert 0 < v.sum()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("method", ["majorityVote", "weightedMajorityVote", "selectFirst", "average",
                                    "weightedAverage", "max", "median"])
@pytest.mark.parametrize("treatment", [None, "skipSegment"])
def test_classification_segmentations(method, treatment):
    plan, s, v, ref, vref = _run(segmented_pmml(method, True, n_segments=6, n_classes=4, seed=11,
                                                missing_treatment=treatment))
    assert (v == vref).all() and v.any()
    assert (s[v] == ref[v]).all()


def test_linear_segment_and_even_median():
    """A RegressionModel segment next to trees; four segments -> even-count medians average the
    two middle values (numpy's rule, not torch.nanmedian's lower middle)."""
    plan, s, v, ref, vref = _run(segmented_pmml("median", False, n_segments=4, seed=5, predicates=False,
                                                linear_segment=True), missing=0.0)
    assert (v == vref).all() and v.all()
    np.testing.assert_allclose(s, ref, rtol=1e-6, atol=1e-6)


def test_true_segment_sums_stay_fused():
    """Plain sum over True tree segments keeps the fused tree kernel."""
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(segmented_pmml("sum", False, predicates=False))
    with lowering_dry_run():
        assert isinstance(compile_plan(c, torch.device("cpu")), TreePlan)


def test_unsupported_segmentation_reason():
    c = CompiledPmml.from_string(segmented_pmml("sum", True, seed=1))  # classification sum: not a PMML rule
    assert "classification multipleModelMethod" in segmentable(c.evaluator, c)


def test_segmented_state_roundtrip():
    from flink_jpmml_amd.runtime.plans import DevicePlan

    c = CompiledPmml.from_string(segmented_pmml("selectFirst", True, seed=2))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
        meta, tensors = plan.export_state()
        q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, torch.device("cpu"))
    assert isinstance(q, SegmentedPlan) and q.n_subs == plan.n_subs and q.progs == plan.progs
    assert [type(a).__name__ for a in q.subs] == [type(b).__name__ for b in plan.subs]
