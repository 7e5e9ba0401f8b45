"""MiningModel ``multipleModelMethod="weightedSum"`` (PMML 4.4, regression): Σ weight_k · value_k
over the segments. Oracle: each segment isolated by zero weights (the Target rescaleConstant of the
synthetic GBDT is added once, after the sum). Device: the regression tree ensemble folds the
weights into the per-tree weights, exactly like weightedAverage without the division. Parity
unpinned (no JPMML here)."""

import re

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml

K = 6


def _weighted(weights) -> str:
    txt = gbdt_pmml(n_trees=K, depth=4, n_features=5, seed=2).replace('multipleModelMethod="sum"',
                                                                     'multipleModelMethod="weightedSum"')
    it = iter(weights)
    out = re.sub(r'<Segment id="(\d+)">', lambda m: f'<Segment id="{m.group(1)}" weight="{next(it)!r}">', txt)
    assert 'weightedSum' in out and out.count('weight="') == K
    return out


def test_weighted_sum_oracle():
    w = [0.5, -1.25, 2.0, 0.0, 3.5, 1.0]
    X = stream_matrix(2000, 5, seed=3, missing_rate=0.05)
    s, v = CompiledPmml.from_string(_weighted(w)).score_matrix_oracle(X)
    expected = np.full(len(X), 0.5)
    for k in range(K):
        sk, vk = CompiledPmml.from_string(_weighted([1.0 if j == k else 0.0 for j in range(K)])).score_matrix_oracle(X)
        assert (vk == v).all()
        expected += w[k] * (sk - 0.5)
    np.testing.assert_allclose(s[v], expected[v], rtol=0, atol=1e-9)


def test_weighted_sum_lowers_to_the_tree_plan():
    from flink_jpmml_amd.runtime.plans import TreePlan, lowering_dry_run

    c = CompiledPmml.from_string(_weighted([0.5, -1.25, 2.0, 0.0, 3.5, 1.0]))
    with lowering_dry_run():
        plan = c.plan("cpu")
    assert isinstance(plan, TreePlan)


@pytest.mark.gpu
def test_weighted_sum_on_gpu(gpu):
    c = CompiledPmml.from_string(_weighted([0.5, -1.25, 2.0, 0.0, 3.5, 1.0]))
    plan = c.plan(gpu)
    X = stream_matrix(20000, 5, seed=4, missing_rate=0.05)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=1e-5)
