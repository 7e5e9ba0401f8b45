"""NearestNeighborModel (``models/knn.py``). Parity unpinned (no JPMML): the oracle is checked
against a per-record brute-force re-implementation of the specification text; k = 1 runs on the
clustering kernel (GPU test)."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import knn_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _wts(d, thr):
    """Weights of the weighted methods; exact matches (zero denominator) alone, equally weighted."""
    d = np.abs(np.asarray(d, dtype=np.float64)) + thr
    exact = d == 0
    if exact.any():
        return exact.astype(np.float64)
    return 1.0 / d


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
        ws = _wts([d[i] for i in order], m.threshold) if m.categorical_method == "weightedMajorityVote" \
            else np.ones(len(order))
        for rank, i in enumerate(order):
            w = ws[rank]
            votes[tgt[i]] = votes.get(tgt[i], 0.0) + w
            first.setdefault(tgt[i], rank)
        best = max(votes.values())
        return float(min((first[t], t) for t, v in votes.items() if v == best)[1])
    y = np.array([float(tgt[i]) for i in order])
    if m.continuous_method == "median":
        return float(np.median(y))
    if m.continuous_method == "weightedAverage":
        w = _wts([d[i] for i in order], m.threshold)
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


# ----------------------------------------------------------------------------- k > 1 on knn.hip

KNN_CASES = [
    # (k, classification, method, metric, measure, compare, target)
    (3, True, "majorityVote", "euclidean", "distance", None, None),
    (7, True, "weightedMajorityVote", "squaredEuclidean", "distance", None, None),
    (5, True, "majorityVote", "cityBlock", "distance", None, None),
    (4, False, "average", "euclidean", "distance", None, None),
    (5, False, "median", "chebychev", "distance", None, None),
    (6, False, "median", "squaredEuclidean", "distance", None, None),
    (8, False, "weightedAverage", 'minkowski p-parameter="3"', "distance", None, None),
    (20, False, "average", "euclidean", "distance", None, 'rescaleFactor="2" rescaleConstant="1" min="-4" max="4"'),
    (12, True, "weightedMajorityVote", "euclidean", "similarity", "gaussSim", None),
    (32, True, "majorityVote", "euclidean", "distance", None, None),
]


def _knn_doc(case, n_instances=300, n_features=6, seed=0):
    k, cls, method, metric, measure, compare, target = case
    return knn_pmml(n_instances=n_instances, n_features=n_features, k=k, classification=cls, method=method,
                    metric=metric, measure=measure, compare=compare, target=target, seed=seed)


def _emulate_knn_kernel(plan, X):
    """numpy model of knn.hip's design: the top-k is chosen on the RAW per-instance sums (the
    Σq/Σq_present rescale and the root are monotone per row), only the k winners are finished."""
    from flink_jpmml_amd.runtime.plans import apply_target_torch

    inst, w, q = plan.inst.numpy().astype(np.float64), plan.weights.numpy().astype(np.float64), plan.qweights.numpy()
    n = X.shape[0]
    pres = ~np.isnan(X)
    diff = np.abs(np.where(pres[:, None, :], X[:, None, :] - inst[None], 0.0))
    m = plan.metric_code
    if plan.similarity:  # gaussSim: exp(-ln2 d² / s²), zero for a missing field
        sc = plan.scales.numpy().astype(np.float64)
        diff = np.where(pres[:, None, :], np.exp(-np.log(2) * diff ** 2 / sc ** 2), 0.0)
    raw = {0: (w * diff ** 2).sum(-1), 1: (w * diff ** 2).sum(-1), 2: (w * diff).sum(-1),
           3: (w * diff).max(-1), 4: (w * diff ** plan.p).sum(-1)}[m]
    key = -raw if plan.similarity else raw
    order = np.argsort(key, axis=1, kind="stable")[:, : plan.k]
    rk = np.take_along_axis(raw, order, axis=1)
    qp = (q * pres).sum(1)
    adj = np.where(qp > 0, q.sum() / np.where(qp > 0, qp, 1), np.nan)[:, None]
    d = rk if m == 3 else rk * adj
    d = np.sqrt(d) if m == 1 else (d ** (1 / plan.p) if m == 4 else d)
    ok = np.isfinite(d).all(1) & (qp > 0)
    if plan.agg < 2:
        cls = plan.inst_class.numpy()[order]
        wt = np.stack([_wts(r, plan.threshold) for r in d]) if plan.agg == 1 else np.ones_like(d)
        votes = np.stack([(wt * (cls == cls[:, [j]])).sum(1) for j in range(plan.k)], 1)
        win = cls[np.arange(n), np.argmax(votes, axis=1)]
        s = plan.class_table.numpy()[win].astype(np.float64)
    else:
        y = plan.inst_value.numpy().astype(np.float64)[order]
        if plan.agg == 2:
            s = y.mean(1)
        elif plan.agg == 3:
            s = np.median(y, 1)
        else:
            wt = np.stack([_wts(r, plan.threshold) for r in d])
            with np.errstate(invalid="ignore"):
                s = (wt * y).sum(1) / wt.sum(1)
    import torch

    st, ot = apply_target_torch(torch.from_numpy(s), torch.from_numpy(ok & np.isfinite(s)), plan.tgt)
    return st.numpy(), ot.numpy()


@pytest.mark.parametrize("case", KNN_CASES, ids=lambda c: f"k{c[0]}-{c[2]}-{c[3].split()[0]}-{c[4]}")
def test_knn_plan_lowering_and_kernel_model(case):
    from flink_jpmml_amd.runtime.plans import KnnPlan, compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(_knn_doc(case))
    with lowering_dry_run():
        plan = compile_plan(c, "cpu")
    assert isinstance(plan, KnnPlan) and plan.k == case[0]
    X = stream_matrix(400, 6, seed=1, missing_rate=0.1).astype(np.float64)
    X[3] = np.nan
    s, v = _emulate_knn_kernel(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("classification,method", [(False, "weightedAverage"), (True, "weightedMajorityVote")])
def test_knn_zero_distance_with_zero_threshold_is_pinned(classification, method):
    """``threshold="0"`` and a query equal to a training instance: ``1/(0 + 0)`` is infinite and
    the weighted average would be inf / inf = NaN. Pinned semantics (parity unpinned, no JPMML):
    the limit as the distance goes to 0 — the exact matches alone, equally weighted. A query
    equal to instance i scores instance i's target (k = 1 behaviour), never NaN / EmptyScore."""
    doc = knn_pmml(n_instances=60, n_features=4, k=5, classification=classification, method=method, seed=3,
                   threshold=0.0, quantum=0.25)
    c = CompiledPmml.from_string(doc)
    m = c.model
    inst = np.array([[float(r[f"c{j}"]) for j in range(4)] for r in m.rows])
    tgt = np.array([float(r["target"]) for r in m.rows])
    uniq = [i for i in range(len(inst)) if (inst == inst[i]).all(axis=1).sum() == 1]
    X = inst[uniq]
    s, v = c.score_matrix_oracle(X)
    assert v.all()
    np.testing.assert_array_equal(s, tgt[uniq])
    for r in range(len(X)):
        assert s[r] == _brute(c, X[r])


def test_knn_targets_applied_by_oracle():
    case = (4, False, "average", "euclidean", "distance", None, 'rescaleFactor="10" rescaleConstant="-3"')
    c1 = CompiledPmml.from_string(_knn_doc(case))
    c0 = CompiledPmml.from_string(_knn_doc(case[:-1] + (None,)))
    X = stream_matrix(50, 6, seed=2).astype(np.float64)
    s1, _ = c1.score_matrix_oracle(X)
    s0, _ = c0.score_matrix_oracle(X)
    np.testing.assert_allclose(s1, s0 * 10 - 3, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["valu", "mfma"])
@pytest.mark.parametrize("case", KNN_CASES, ids=lambda c: f"k{c[0]}-{c[2]}-{c[3].split()[0]}-{c[4]}")
def test_knn_kernel_matches_oracle(gpu, case, variant):
    from flink_jpmml_amd.runtime.plans import KnnPlan, NotLowerable

    c = CompiledPmml.from_string(_knn_doc(case, n_instances=700, n_features=12, seed=5))
    try:
        plan = c.plan(gpu, knn_variant=variant)
    except NotLowerable:
        assert variant == "mfma" and (case[3] not in ("euclidean", "squaredEuclidean") or case[4] != "distance")
        return
    assert isinstance(plan, KnnPlan) and plan.variant == variant
    X = stream_matrix(20_000, 12, seed=6, missing_rate=0.03)
    X[:300, 1:] = np.nan  # rows with few present fields: rescaled exact path
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).mean() > 0.999
    both = v & vref
    close = np.isclose(s[both], ref[both], rtol=1e-4, atol=1e-5)
    # fp32 distances may swap two neighbours the fp64 oracle ranks a hair apart
    assert close.mean() > 0.998, close.mean()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["valu", "mfma"])
@pytest.mark.parametrize("classification,method", [(False, "weightedAverage"), (True, "weightedMajorityVote")])
def test_knn_kernel_zero_distance_zero_threshold(gpu, variant, classification, method):
    """The kernel applies the same pinned exact-match rule as the oracle (no NaN for d = 0)."""
    from flink_jpmml_amd.runtime.plans import NotLowerable

    doc = knn_pmml(n_instances=500, n_features=8, k=6, classification=classification, method=method, seed=4,
                   threshold=0.0, quantum=0.25, metric="euclidean")
    c = CompiledPmml.from_string(doc)
    try:
        plan = c.plan(gpu, knn_variant=variant)
    except NotLowerable:
        pytest.skip(f"{variant} does not lower this model")
    m = c.model
    inst = np.array([[float(r[f"c{j}"]) for j in range(8)] for r in m.rows], dtype=np.float32)
    X = np.concatenate([inst, stream_matrix(2000, 8, seed=2)]).astype(np.float32)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    n0 = len(inst)
    assert v[:n0].all() and vref[:n0].all()
    np.testing.assert_allclose(s[:n0], ref[:n0], rtol=1e-5, atol=1e-6)  # the exact matches
    both = v & vref
    assert (v == vref).mean() > 0.999
    assert np.isclose(s[both], ref[both], rtol=1e-4, atol=1e-5).mean() > 0.998
