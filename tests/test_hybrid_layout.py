"""HYBRID tree layout (deep forests: PERFECT head in LDS + POINTER tail from L2,
``ops/csrc/tree_hybrid.hip``) and the vectorised POINTER packer: a numpy emulation of the kernel
walk over the packed tensors reproduces the float64 oracle (CPU, dry-run plans)."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import TB, TreePlan, lowering_dry_run


def _plan(txt, **kw):
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        return c, TreePlan(c, torch.device("cpu"), **kw)


def _feature(X, meta, feat_lds):
    f = (meta & 0xFFFF) // (TB * 4) if feat_lds else (meta & 0xFFFF)
    return X[np.arange(len(X)), f]


def emulate(plan, X):
    """Per-row accumulator (P = 1) of the hybrid / pointer kernel, NaN where the row is poisoned."""
    Xf = X.astype(np.float32)
    n = len(X)
    feat_lds = plan.n_features <= 64
    H = plan.head_depth
    if plan.variant == 32:
        return emulate_compact(plan, Xf)
    compact_tail = bool(H) and getattr(plan, "tail_format", 0) == 0
    tail = plan.blob.numpy().view(np.uint32).reshape(-1, 2 if compact_tail else 4)
    leaves = plan.leaves.numpy().reshape(-1, plan.P)[:, 0]
    NI = (1 << H) - 1
    acc = np.zeros(n)
    heads = plan.heads.numpy().view(np.uint32).reshape(plan.n_trees, -1) if H else None
    for t in range(plan.n_trees):
        pz = np.zeros(n, bool)
        if H:
            rec = heads[t]
            j = np.zeros(n, np.int64)
            for _ in range(H):
                T = rec[2 * j].view(np.float32)
                meta = rec[2 * j + 1]
                x = _feature(Xf, meta, feat_lds)
                isn = np.isnan(x)
                pz |= isn & ((meta >> 30) & 1).astype(bool)
                right = (x >= T) | (isn & (meta >> 31).astype(bool))
                j = 2 * j + 1 + right
            code = rec[2 * NI + (j - NI)].view(np.int32).astype(np.int64)
        else:
            code = np.full(n, plan.roots.numpy()[t], np.int64)
        if compact_tail:  # COMPACT depth-first tail: left child adjacent, right at +rel, stop at the leaf's parent
            done = pz | (code < 0)
            code = np.where(code < 0, ~code, code)
            while (~done).any():
                nd = tail[code]
                act = ~done
                f = nd[:, 1] & 0xFF
                x = Xf[np.arange(n), f]
                isn = np.isnan(x)
                nulled = act & isn & ((nd[:, 1] >> 30) & 1).astype(bool)
                right = (x >= nd[:, 0].view(np.float32)) | (isn & (nd[:, 1] >> 31).astype(bool))
                nxt = np.where(right, code + ((nd[:, 1] >> 8) & 0xFFFFF), code + 1)
                child_leaf = np.where(right, (nd[:, 1] >> 28) & 1, (nd[:, 1] >> 29) & 1).astype(bool)
                pz |= nulled
                code = np.where(act & ~nulled, nxt, code)
                done |= nulled | child_leaf
            val = tail[code, 0]
            lv = leaves[val] if plan.P > 1 else val.view(np.float32)
            acc += np.where(pz, np.nan, lv)
            continue
        code = np.where(pz, -1, code)
        while (code >= 0).any():
            act = code >= 0
            nd = tail[np.maximum(code, 0)]
            x = _feature(Xf, nd[:, 1], feat_lds)
            isn = np.isnan(x)
            nulled = act & isn & ((nd[:, 1] >> 30) & 1).astype(bool)
            right = (x >= nd[:, 0].view(np.float32)) | (isn & (nd[:, 1] >> 31).astype(bool))
            nc = np.where(right, nd[:, 3].view(np.int32), nd[:, 2].view(np.int32)).astype(np.int64)
            pz |= nulled
            code = np.where(act, np.where(nulled, -1, nc), code)
        acc += np.where(pz, np.nan, leaves[np.where(pz, 0, ~code)])
    return acc


def emulate_compact(plan, Xf):
    """The 8-byte BFS pointer kernel (``tree_compact_kernel``): children at first, first + 1;
    the walk stops on a leaf's parent and reads the leaf slot's x."""
    n = len(Xf)
    nodes = plan.blob.numpy().view(np.uint32).reshape(-1, 2)
    leaves = plan.leaves.numpy().reshape(-1, plan.P)[:, 0]
    acc = np.zeros(n)
    for t in range(plan.n_trees):
        r = int(plan.roots.numpy()[t])
        pos = np.full(n, r if r >= 0 else ~r, np.int64)
        act = np.full(n, r >= 0)
        pz = np.zeros(n, bool)
        while act.any():
            nd = nodes[np.where(act, pos, 0)]
            m = nd[:, 1]
            x = Xf[np.arange(n), m & 63]
            isn = np.isnan(x)
            nulled = act & isn & ((m >> 30) & 1).astype(bool)
            right = (x >= nd[:, 0].view(np.float32)) | (isn & (m >> 31).astype(bool))
            child = pos + ((m >> 8) & 0x3FFFFF) + right
            leaf = np.where(right, (m >> 7) & 1, (m >> 6) & 1).astype(bool)
            pz |= nulled
            pos = np.where(act & ~nulled, child, pos)
            act = act & ~nulled & ~leaf
        val = nodes[pos, 0]
        lv = leaves[val] if plan.P > 1 else val.view(np.float32)
        acc += np.where(pz, np.nan, lv)
    return acc


@pytest.mark.parametrize("layout,head,fmt", [("hybrid", 8, "auto"), ("hybrid", 4, "auto"), ("hybrid", 10, "auto"),
                                             ("pointer", 0, "compact"), ("pointer", 0, "wide")])
@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
def test_deep_regression_forest_layouts_match_oracle(layout, head, fmt, missing):
    txt = gbdt_pmml(n_trees=12, depth=13, n_features=20, seed=3, p_split=0.8)
    if missing == "nullPrediction":
        txt = txt.replace('missingValueStrategy="defaultChild"', 'missingValueStrategy="nullPrediction"')
    c, plan = _plan(txt, layout=layout, head_depth=head, node_format=fmt)
    assert plan.layout == layout and plan.head_depth == head
    assert (plan.variant == 32) == (fmt == "compact")
    X = stream_matrix(4000, 20, seed=5, missing_rate=0.03)
    ref, vref = c.score_matrix_oracle(X)
    out = emulate(plan, X)
    a, b = plan.epi_args.get("a", 1.0), plan.epi_args.get("b", 0.0)
    got = a * out + b
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-4)


def test_auto_layout_picks_pointer_for_deep_forests():
    """Deeper than the PERFECT layout's 10 levels -> the pointer walk (profiles/r3q: faster than
    the hybrid head on 300 x depth-14 forests); the hybrid layout stays available on request."""
    c, plan = _plan(random_forest_pmml(n_trees=6, depth=14, n_features=16, n_classes=3, seed=2))
    assert plan.layout == "pointer" and plan.head_depth == 0 and plan.xcd_split == 0
    assert plan.general == 1  # class votes accumulate in LDS slots
    _, hyb = _plan(random_forest_pmml(n_trees=6, depth=14, n_features=16, n_classes=3, seed=2), layout="hybrid")
    assert hyb.layout == "hybrid" and hyb.head_depth == 4 and hyb.chunk_trees >= 1


def test_xcd_split_option():
    """XCD tree slices: opt-in, 8 slices (one per XCD) once the forest has >= 16 trees."""
    txt = gbdt_pmml(n_trees=20, depth=12, n_features=8, seed=2, p_split=0.7)
    _, on = _plan(txt, layout="pointer", xcd_split="on")
    _, off = _plan(txt, layout="pointer")
    assert on.xcd_split == 8 and on._auto_splits(1 << 20) == 8
    assert off.xcd_split == 0 and off._auto_splits(1 << 20) == 1
    with pytest.raises(ValueError):
        _plan(txt, layout="pointer", xcd_split="maybe")


def test_shallow_trees_and_stumps_in_the_head():
    """Trees shallower than the head (and a single-leaf stump) route through padding nodes."""
    txt = gbdt_pmml(n_trees=9, depth=5, n_features=6, seed=11, p_split=0.6)
    c, plan = _plan(txt, layout="hybrid", head_depth=8)
    X = stream_matrix(3000, 6, seed=1, missing_rate=0.05)
    ref, vref = c.score_matrix_oracle(X)
    got = plan.epi_args.get("a", 1.0) * emulate(plan, X) + plan.epi_args.get("b", 0.0)
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-5)


def test_wide_feature_pointer_offsets():
    """n_features > 64: features stay in global memory; metas hold indices (the old packer wrote
    LDS byte offsets for features < 64 there)."""
    txt = gbdt_pmml(n_trees=5, depth=12, n_features=90, seed=4)
    c, plan = _plan(txt, layout="pointer")
    meta = plan.blob.numpy().view(np.uint32).reshape(-1, 4)[:, 1] & 0xFFFF
    assert meta.max() < 90
    X = stream_matrix(1500, 90, seed=2, missing_rate=0.02)
    ref, vref = c.score_matrix_oracle(X)
    got = plan.epi_args.get("a", 1.0) * emulate(plan, X) + plan.epi_args.get("b", 0.0)
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-4)


def emulate_super(plan, X):
    """``tree_super_kernel`` over the packed super-node slots: per step x_j picks the child, x_c the
    grandchild slot ``base + 1 + 4 * block + 2 (c == r) + (x_c >= T_c)``."""
    Xf = X.astype(np.float32)
    n = len(X)
    nodes = plan.blob.numpy().view(np.uint32).reshape(-1, 4)
    roots = plan.roots.numpy().view(np.uint32)
    leaves = plan.leaves.numpy().reshape(-1, plan.P)[:, 0]
    rows = np.arange(n)
    acc = np.zeros(n)
    for t in range(plan.n_trees):
        base = int(roots[t] & 0x7FFFFFFF)
        nul = bool(roots[t] >> 31)
        pos = np.full(n, base)
        act = np.ones(n, bool)
        pz = np.zeros(n, bool)
        leafv = np.zeros(n, np.uint32)
        while act.any():
            nd = nodes[np.where(act, pos, 0)]
            m = nd[:, 3]
            self_leaf = (m & (1 << 17)) != 0
            xj = Xf[rows, m & 31]
            nj = np.isnan(xj)
            r1 = (xj >= nd[:, 0].view(np.float32)) | (nj & ((m >> 18) & 1).astype(bool))
            tc = np.where(r1, nd[:, 2], nd[:, 1])
            fc = np.where(r1, (m >> 10) & 31, (m >> 5) & 31)
            cleaf = np.where(r1, (m >> 16) & 1, (m >> 15) & 1).astype(bool)
            drc = np.where(r1, (m >> 20) & 1, (m >> 19) & 1).astype(bool)
            xc = Xf[rows, fc]
            nc = np.isnan(xc)
            r2 = (xc >= tc.view(np.float32)) | (nc & drc)
            nulled = act & ~self_leaf & nul & (nj | (~cleaf & nc))
            done = self_leaf | cleaf
            leafv = np.where(act, np.where(self_leaf, nd[:, 0], np.where(cleaf, tc, leafv)), leafv)
            pz |= nulled
            nxt = base + 1 + 4 * (m >> 21).astype(np.int64) + 2 * r1 + r2
            pos = np.where(act & ~done, nxt, pos)
            act = act & ~done & ~nulled
        lv = leaves[leafv] if plan.P > 1 else leafv.view(np.float32)
        acc += np.where(pz, np.nan, lv)
    return acc


@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
@pytest.mark.parametrize("depth,p_split", [(13, 0.8), (5, 0.6), (16, 0.75)])
def test_super_layout_matches_oracle(missing, depth, p_split):
    txt = gbdt_pmml(n_trees=10, depth=depth, n_features=20, seed=7, p_split=p_split)
    if missing == "nullPrediction":
        txt = txt.replace('missingValueStrategy="defaultChild"', 'missingValueStrategy="nullPrediction"')
    c, plan = _plan(txt, layout="pointer", node_format="super")
    assert plan.variant == 128
    X = stream_matrix(3000, 20, seed=5, missing_rate=0.03)
    ref, vref = c.score_matrix_oracle(X)
    got = plan.epi_args.get("a", 1.0) * emulate_super(plan, X) + plan.epi_args.get("b", 0.0)
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-4)


def test_super_layout_votes_and_limits():
    txt = random_forest_pmml(n_trees=5, depth=12, n_features=16, n_classes=3, seed=4, p_split=0.8)
    c, plan = _plan(txt, layout="pointer", node_format="super")
    assert plan.variant == 128 and plan.P == 3
    nodes = plan.blob.numpy().view(np.uint32).reshape(-1, 4)
    roots = plan.roots.numpy().view(np.uint32)
    assert (roots >> 31 == 0).all() and int(roots.max()) < len(nodes)
    from flink_jpmml_amd.runtime.plans import NotLowerable

    with pytest.raises(NotLowerable):  # 5-bit feature fields
        _plan(gbdt_pmml(n_trees=3, depth=6, n_features=40, seed=1), layout="pointer", node_format="super")


@pytest.mark.parametrize("H", [2, 3, 4])
@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
def test_hybrid_wide_tail_emulation_matches_oracle(H, missing):
    """LDS head + 16-byte BFS pointer tail (``tree_hybrid_ptr_kernel``): head exits are pointer
    codes (tail node index or ~leaf) into :func:`pack_trees`' tail."""
    txt = gbdt_pmml(n_trees=12, depth=12, n_features=20, seed=3, p_split=0.8, missing_strategy=missing)
    c, plan = _plan(txt, layout="hybrid", hybrid_tail="wide", head_depth=H)
    assert plan.layout == "hybrid" and plan.tail_format == 1 and plan.head_depth == H
    with lowering_dry_run():
        assert TreePlan(c, torch.device("cpu"), layout="hybrid", hybrid_tail="wide", head_depth=H,
                        pointer_load="uskip").tail_format == 2
    X = stream_matrix(3000, 20, seed=2, missing_rate=0.05)
    ref, vref = c.score_matrix_oracle(X)
    got = plan.epi_args.get("a", 1.0) * emulate(plan, X) + plan.epi_args.get("b", 0.0)
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-5)


def test_hybrid_wide_tail_rejects_bad_head_depth():
    txt = gbdt_pmml(n_trees=4, depth=8, n_features=8, seed=1)
    with pytest.raises(ValueError):
        _plan(txt, layout="hybrid", hybrid_tail="compact", head_depth=3)
    with pytest.raises(ValueError):
        _plan(txt, layout="hybrid", hybrid_tail="wide", head_depth=5)
    with pytest.raises(ValueError):
        _plan(txt, layout="pointer", pointer_load="bogus")
