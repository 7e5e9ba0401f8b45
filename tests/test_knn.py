"""NearestNeighborModel (``models/knn.py``). Parity unpinned (no JPMML): the oracle is checked
against a per-record brute-force re-implementation of the specification text; k = 1 runs on the
clustering kernel (GPU test)."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import knn_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _brute(c, x):
    m = c.model
    inst = np.array([[float(r[f"c{j}"]) for j in range(len(m.inputs))] for r in m.rows])
    tgt = [r["target"] for r in m.rows]
    pres = ~np.isnan(x)
    d2 = ((inst[:, pres] - x[pres]) ** 2).sum(axis=1) * (len(x) / pres.sum())
    d = np.sqrt(d2)
    order = sorted(range(len(d)), key=lambda i: (d[i], i))[: m.k]
    if m.function_name == "classification":
        votes, first = {}, {}
        for rank, i in enumerate(order):
            w = 1.0 / (d[i] + m.threshold) if m.categorical_method == "weightedMajorityVote" else 1.0
            votes[tgt[i]] = votes.get(tgt[i], 0.0) + w
            first.setdefault(tgt[i], rank)
        best = max(votes.values())
        return float(min((first[t], t) for t, v in votes.items() if v == best)[1])
    y = np.array([float(tgt[i]) for i in order])
    if m.continuous_method == "median":
        return float(np.median(y))
    if m.continuous_method == "weightedAverage":
        w = np.array([1.0 / (d[i] + m.threshold) for i in order])
        return float((w * y).sum() / w.sum())
    return float(y.mean())


@pytest.mark.parametrize("k,classification,method", [(1, True, None), (3, True, None), (5, True, "weightedMajorityVote"),
                                                     (4, False, "average"), (3, False, "median"),
                                                     (6, False, "weightedAverage")])
def test_knn_matches_brute_force(k, classification, method):
    c = CompiledPmml.from_string(knn_pmml(n_instances=150, k=k, classification=classification, method=method, seed=k))
    X = stream_matrix(300, 4, seed=k, missing_rate=0.1).astype(np.float64)
    s, v = c.score_matrix_oracle(X)
    for r in range(len(X)):
        if np.isnan(X[r]).all():
            assert not v[r]
            continue
        assert v[r]
        assert abs(s[r] - _brute(c, X[r])) < 1e-9


@pytest.mark.gpu
def test_knn_k1_on_cluster_kernel(gpu):
    from flink_jpmml_amd.runtime.plans import ClusterPlan

    c = CompiledPmml.from_string(knn_pmml(n_instances=512, n_features=16, k=1, metric="squaredEuclidean", seed=3))
    plan = c.plan(gpu)
    assert isinstance(plan, ClusterPlan) and plan.variant == "mfma"
    X = stream_matrix(20_000, 16, seed=4, missing_rate=0.02)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.999
