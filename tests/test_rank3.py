"""RANK3 pointer layout (three tree levels per 16-byte record on per-feature threshold ranks,
VERDICT r3 item 3): the packer's records, walked by a numpy model of ``tree_rank3_kernel``,
reproduce a direct walk of the canonical trees exactly (same leaves, same order); the GPU kernel
is checked bit-for-bit against the 16-byte pointer walk in tests/test_gpu_rank3.py."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.hybrid import RK_NAN, pack_rank3
from flink_jpmml_amd.runtime.plans import _canonical_vec, ensemble_spec


def walk_rank3(nodes, roots, thr, cnt, X, P=1, leaves=None):
    """numpy model of tree_rank3_kernel: per row, ranks by upper_bound, then record walks."""
    n, F = X.shape
    rk = np.full((n, F), RK_NAN, dtype=np.int64)
    for f in range(F):
        t = thr[f, : cnt[f]]
        ok = ~np.isnan(X[:, f])
        rk[ok, f] = np.searchsorted(t, X[ok, f], side="right")
    lo = nodes[:, 0].astype(np.uint64) | (nodes[:, 1].astype(np.uint64) << np.uint64(32))
    hi = nodes[:, 2].astype(np.uint64) | (nodes[:, 3].astype(np.uint64) << np.uint64(32))
    out = np.zeros((n, P), dtype=np.float32)
    rows = np.arange(n)
    for base in roots.astype(np.int64):
        pos = np.full(n, base, dtype=np.int64)
        act = np.ones(n, dtype=bool)
        leafv = np.zeros(n, dtype=np.uint32)
        while act.any():
            l_, h_ = lo[pos], hi[pos]
            leaf = (h_ >> np.uint64(63)) != 0
            done = act & leaf
            leafv[done] = nodes[pos[done], 0]

            fsh = np.array([0, 5, 10, 15, 20, 25, 32], dtype=np.uint64)
            dsh = np.array([30, 31, 37, 38, 39, 40, 41], dtype=np.uint64)

            def right(nn):
                f = ((h_ >> fsh[nn]) & np.uint64(31)).astype(np.int64)
                r = ((l_ >> (np.uint64(8) * nn.astype(np.uint64))) & np.uint64(255)).astype(np.int64)
                d = ((h_ >> dsh[nn]) & np.uint64(1)).astype(np.int64)
                k = rk[rows, f]
                return np.where(k == RK_NAN, d, (k >= r).astype(np.int64))

            b0 = right(np.zeros(n, np.int64))
            b1 = right(1 + b0)
            b2 = right(3 + 2 * b0 + b1)
            e = 4 * b0 + 2 * b1 + b2
            mask = ((l_ >> np.uint64(56)) & np.uint64(255)).astype(np.int64) & ((1 << e) - 1)
            below = np.array([bin(m).count("1") for m in mask], dtype=np.int64)
            nxt = base + ((h_ >> np.uint64(42)) & np.uint64(0x1FFFFF)).astype(np.int64) + below
            go = act & ~leaf
            pos = np.where(go, nxt, pos)
            act = go
        if P == 1:
            out[:, 0] += leafv.view(np.float32)
        else:
            out += leaves[leafv.astype(np.int64)]
    return out


def walk_direct(spec, X):
    """The canonical trees walked node by node ("go right iff x >= T", default direction on NaN)."""
    out = np.zeros((X.shape[0], spec.P), dtype=np.float32)
    for t, w in zip(spec.trees, spec.weights):
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        lc = np.where(swap, t.right, t.left)
        rc = np.where(swap, t.left, t.right)
        dr = np.where(swap, np.asarray(t.default_left, bool), ~np.asarray(t.default_left, bool))
        node = np.zeros(X.shape[0], dtype=np.int64)
        rows = np.arange(X.shape[0])
        while True:
            inner = np.asarray(t.feature)[node] >= 0
            if not inner.any():
                break
            f = np.where(inner, np.asarray(t.feature)[node], 0)
            x = X[rows, f]
            go_r = np.where(np.isnan(x), dr[node], x >= T[node])
            node = np.where(inner, np.where(go_r, rc[node], lc[node]), node)
        if spec.P == 1:
            out[:, 0] += (np.asarray(t.leaf_value, dtype=np.float64)[node] * w).astype(np.float32)
        else:
            out += (np.asarray(t.leaf_probs, dtype=np.float64)[node, : spec.P] * w).astype(np.float32)
    return out


@pytest.mark.parametrize("depth,p_split", [(3, 1.0), (7, 0.85), (12, 0.85)])
def test_rank3_records_walk_like_the_trees(depth, p_split):
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=12, depth=depth, n_features=16, seed=depth, p_split=p_split))
    spec = ensemble_spec(c)
    nodes, leaves, roots, thr, cnt, has_dr = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features)
    # footprint: about the 16-byte pointer layout's (nodes x 16 B + leaves x 4 B), at 3 levels a fetch
    n_int = sum(int((np.asarray(t.feature) >= 0).sum()) for t in spec.trees)
    n_leaf = sum(len(t.feature) for t in spec.trees) - n_int
    assert nodes.shape[0] * 16 <= 3.0 * (n_int * 16 + n_leaf * 4)
    X = stream_matrix(3000, c.n_features, seed=1, missing_rate=0.1).astype(np.float32)
    X[:5] = np.inf
    X[5:10] = -np.inf
    got = walk_rank3(nodes, roots, thr, cnt, X)
    # same leaves in the same tree order: compare per-tree leaf sums through the direct walk
    ref = walk_direct(spec, X)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5)


def test_rank3_multiclass_leaf_rows():
    c = CompiledPmml.from_string(random_forest_pmml(n_trees=8, depth=6, n_features=12, n_classes=3, seed=2))
    spec = ensemble_spec(c)
    if spec.P == 1:
        pytest.skip("vote forest packs scalar leaves")
    nodes, leaves, roots, thr, cnt, _ = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features)
    X = stream_matrix(1000, c.n_features, seed=3, missing_rate=0.05).astype(np.float32)
    np.testing.assert_allclose(walk_rank3(nodes, roots, thr, cnt, X, spec.P, leaves), walk_direct(spec, X),
                               rtol=0, atol=1e-5)


def test_rank3_refuses_too_many_thresholds():
    from flink_jpmml_amd.runtime.hybrid import rank_tables

    class T:
        feature = np.zeros(600, dtype=np.int64)
        op = np.zeros(600, dtype=np.int64)
        threshold = np.linspace(-1, 1, 600)
        left = right = default_left = np.zeros(600, dtype=np.int64)

    with pytest.raises(ValueError, match="unique thresholds"):
        rank_tables([T()], 1)


def test_rank3_plan_lowers_and_roundtrips():
    from flink_jpmml_amd.runtime.plans import DevicePlan, TreePlan, compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=6, depth=9, n_features=16, seed=3, p_split=0.85))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"), layout="pointer", node_format="rank3")
        assert isinstance(plan, TreePlan) and plan.variant == 1024 and plan.rank_stride >= 1
        meta, tensors = plan.export_state()
        q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, torch.device("cpu"))
    assert q.variant == 1024 and torch.equal(q.rank_thr, plan.rank_thr) and q.rank_stride == plan.rank_stride


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gbdt", "rf"])
@pytest.mark.parametrize("ilp", [4, 8, 16])
def test_rank3_kernel_bit_identical_to_pointer_walk(gpu, model, ilp):
    """tree_rank3_kernel reaches the same leaves in the same tree order as the 16-byte pointer walk:
    identical bits, validity and (for the vote forest) labels, with missing values and +-inf."""
    if model == "gbdt":
        doc = gbdt_pmml(n_trees=40, depth=12, n_features=32, seed=5, p_split=0.85)
    else:
        doc = random_forest_pmml(n_trees=40, depth=12, n_features=32, n_classes=3, seed=5)
    c = CompiledPmml.from_string(doc)
    X = stream_matrix(30_001, 32, seed=8, missing_rate=0.05)
    X[:7] = np.inf
    X[7:14] = -np.inf
    ref_plan = c.plan(gpu, layout="pointer")
    plan = c.plan(gpu, layout="pointer", node_format="rank3", pointer_ilp=ilp)
    assert plan.variant == 1024
    s0, v0 = ref_plan.score(X)
    s1, v1 = plan.score(X)
    assert torch.equal(v0, v1)
    m = v0.bool()
    assert torch.equal(s0[m].view(torch.int32), s1[m].view(torch.int32))
    ref, vref = c.score_matrix_oracle(X)
    assert (v1.cpu().numpy().astype(bool) == vref).all()


@pytest.mark.parametrize("depth,p_split,seed", [(12, 0.85, 1), (3, 1.0, 2), (9, 0.7, 3)])
def test_vectorized_packer_matches_reference_builder(depth, p_split, seed):
    """The level-at-a-time numpy packer (default) emits exactly the record-by-record builder's
    slots, leaves, roots and rank tables."""
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=10, depth=depth, n_features=24, seed=seed, p_split=p_split))
    spec = ensemble_spec(c)
    a = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features, vectorized=False)
    b = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features, vectorized=True)
    for x, y in zip(a, b):
        assert (x is None and y is None) or np.array_equal(x, y)


def test_vectorized_packer_multislot_leaves():
    """P > 1 leaf rows (the pointer layout's vote / probability forests): identical leaf tables."""
    from flink_jpmml_amd.runtime.plans import TreePlan, lowering_dry_run

    c = CompiledPmml.from_string(random_forest_pmml(n_trees=12, depth=9, n_features=20, n_classes=3, seed=5))
    with lowering_dry_run():
        plan = TreePlan(c, torch.device("cpu"), layout="pointer", node_format="rank3")
    spec = plan.spec
    a = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features, vectorized=False)
    b = pack_rank3(spec.trees, spec.weights, spec.P, c.n_features, vectorized=True)
    assert spec.P > 1 and a[1].shape[1] == spec.P
    for x, y in zip(a, b):
        assert (x is None and y is None) or np.array_equal(x, y)
    X = stream_matrix(2000, c.n_features, seed=3, missing_rate=0.05).astype(np.float32)
    np.testing.assert_allclose(walk_rank3(b[0], b[2], b[3], b[4], X, spec.P, b[1]), walk_direct(spec, X),
                               rtol=0, atol=1e-5)
