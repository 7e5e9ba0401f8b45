"""CPU emulation of the wide PERFECT tree kernel (csrc/tree_common.h ``tree_perfect_wide_kernel``)
over the tensors a real :class:`TreePlan` lowers to (``lowering_dry_run``: no GPU, no HIP library):
feature planes of stride ``rows``, staged-column compaction (``feat_map``), the NaN -> +inf
second plane, and the four accumulation modes (SUM, SLOT for K-class GBDT chains, CLASS for
weighted votes, VOTE8 for packed u8 vote counters). Each must reproduce the float64 oracle.

Parity: the K-class chain mirrors the XGBoost multi:softprob export the reference scores through
JPMML (reference ``flink-jpmml-scala/src/test/resources`` models are binary / regression only —
parity unpinned for K > 2 beyond the oracle)."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import VAR_NAN_FAST, VAR_NAN_PLANES, TreePlan, lowering_dry_run


def _plan(txt, **kw):
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        return c, TreePlan(c, torch.device("cpu"), **kw)


def emulate_wide(plan, X, use_nan_blob):
    """Per-row result of the wide kernel; ``use_nan_blob`` picks the tile path (NaN blob + two
    planes, as for a tile with missing values) — without it missing values take the per-node
    default-right bits (traverse_chunk_g)."""
    D, n_t, rec = plan.depth, plan.n_trees, plan.rec_words
    NI, NL = (1 << D) - 1, 1 << D
    PS = plan.rows_wide
    G = 1024 // plan.rows_wide
    stage = plan.feat_map.numpy() if plan.feat_map is not None else np.arange(plan.n_features)
    Xs = X[:, stage].astype(np.float32)
    Fs = Xs.shape[1]
    blob = (plan.blob_nan if use_nan_blob else plan.blob).numpy().view(np.uint32).reshape(n_t, rec)
    planes = np.concatenate([Xs, np.where(np.isnan(Xs), np.float32(np.inf), Xs)], axis=1) if use_nan_blob else Xs
    chunk = plan.chunk_trees_nan if use_nan_blob else plan.chunk_trees
    per_node = not use_nan_blob and not (plan.variant & VAR_NAN_FAST)
    n = len(X)
    rows = np.arange(n)
    C = plan.C
    acc = np.zeros((n, max(C, 1)), np.float64)
    votes = np.zeros((G, n, 4), np.int64)
    pz = np.zeros(n, bool)
    slots = plan.slots.numpy() if plan.slots is not None else None
    tree_w = plan.tree_w.numpy() if plan.tree_w is not None else np.ones(n_t, np.float32)
    for t in range(n_t):
        T = blob[t, 0:2 * NI:2].view(np.float32)
        meta = blob[t, 1:2 * NI:2]
        codes = plan.variant & 3 == 2  # VOTE8 class codes in the last-level metas (no leaf array)
        leaves = None if codes else blob[t, 2 * NI:2 * NI + NL]
        drw = blob[t, 2 * NI + (0 if codes else NL):2 * NI + (0 if codes else NL) + (NI + 31) // 32]
        j = np.ones(n, np.int64)
        miss = np.zeros(n, bool)
        for lev in range(D):
            off = meta[j - 1].astype(np.int64) & (0xFFFF if codes and lev == D - 1 else 0xFFFFFFFF)
            assert (off % (PS * 4) == 0).all()
            x = planes[rows, off // (PS * 4)]
            right = x >= T[j - 1]
            if per_node:
                isn = np.isnan(x)
                right |= isn & (((drw[(j - 1) >> 5] >> ((j - 1) & 31)) & 1) == 1)
                miss |= isn
            j = 2 * j + right
        null_tree = (drw[NI >> 5] >> (NI & 31)) & 1
        if codes:
            pm = meta[(j >> 1) - 1]
            lv = np.uint32(1) << (np.uint32(8) * ((pm >> np.where(j & 1, 24, 16).astype(np.uint32)) & 3))
        else:
            lv = leaves[j - NL]
        poison = miss & (null_tree == 1)
        if plan.mode == 0:
            acc[:, 0] += np.where(poison, np.nan, lv.view(np.float32))
        elif plan.mode == 1:
            acc[~poison, slots[t]] += lv.view(np.float32)[~poison]
        elif plan.mode == 2:
            v = lv.view(np.float32)
            pz |= poison | np.isnan(v)
            ok = ~poison & ~np.isnan(v)
            acc[rows[ok], v[ok].astype(int)] += tree_w[t]
        else:
            g = (t % chunk) % G
            for k in range(4):
                votes[g, ~poison, k] += (lv[~poison] >> (8 * k)) & 0xFF
        pz |= poison
    if plan.mode == 3:
        assert votes.max() <= 255  # a thread's packed u8 counter never carries
        acc = votes.sum(axis=0)[:, :C].astype(np.float64)
    if plan.acc_init is not None:
        acc += plan.acc_init.numpy()[None, :]
    tab = np.array([float(x) for x in plan.labels]) if plan.labels is not None else None
    e = plan.epi_args
    if plan.mode == 0 and e["mode"] == 0:
        return np.where(np.isnan(acc[:, 0]), np.nan, e["a"] * acc[:, 0] + e["b"])
    if plan.mode == 0 and e["mode"] == 1:
        p0 = 1.0 / (1.0 + np.exp(-(e["a"] * acc[:, 0] + e["b"])))
        return np.where(np.isnan(acc[:, 0]), np.nan, tab[np.where(p0 >= 0.5, 0, 1)])
    return np.where(pz, np.nan, tab[np.argmax(acc, axis=1)])  # argmax: ties -> lowest class


def _check(c, plan, X, tol=0.0):
    ref, vref = c.score_matrix_oracle(X)
    paths = [False] + ([True] if plan.blob_nan is not None else [])
    for use_nan in paths:
        # with a NaN blob, the main blob only ever sees tiles without missing values
        stage = plan.feat_map.numpy() if plan.feat_map is not None else np.arange(X.shape[1])
        keep = ~np.isnan(X[:, stage]).any(axis=1) if plan.blob_nan is not None and not use_nan \
            else np.ones(len(X), bool)
        if not keep.any():
            continue
        out, r, vr = emulate_wide(plan, X[keep], use_nan), ref[keep], vref[keep]
        assert (np.isfinite(out) == vr).all(), use_nan
        if tol:
            assert np.max(np.abs(out[vr] - r[vr])) < tol
        else:
            agree = (out[vr] == r[vr]).mean()
            assert agree == 1.0, (use_nan, agree)
    return paths


@pytest.mark.parametrize("K", [3, 5, 8])
def test_multiclass_chain_slot_mode(K):
    c, plan = _plan(gbdt_pmml(n_trees=12, depth=5, n_features=10, objective="multiclass", n_classes=K, seed=K))
    assert plan.layout == "perfect" and plan.variant & 3 == 1 and plan.mode == 1 and plan.C == K
    assert plan.acc_init is not None  # per-class intercepts start the accumulators
    X = stream_matrix(2500, 10, seed=K, missing_rate=0.05)
    assert _check(c, plan, X) == [False, True]  # default-right nodes: NaN planes


def test_multiclass_chain_nine_classes_stays_general():
    c, plan = _plan(gbdt_pmml(n_trees=4, depth=3, n_features=6, objective="multiclass", n_classes=9))
    assert plan.mode == 0 and (plan.layout == "pointer" or plan.general)


def test_unweighted_forest_uses_vote8():
    c, plan = _plan(random_forest_pmml(n_trees=40, depth=6, n_features=12, n_classes=3, seed=1))
    assert plan.mode == 3 and plan.variant & 3 == 2  # class codes in the last-level metas
    _check(c, plan, stream_matrix(3000, 12, seed=2, missing_rate=0.04))


def test_forest_many_classes_uses_class_mode():
    c, plan = _plan(random_forest_pmml(n_trees=30, depth=5, n_features=12, n_classes=6, seed=3))
    assert plan.mode == 2 and plan.C == 6
    _check(c, plan, stream_matrix(3000, 12, seed=4, missing_rate=0.04))


def test_null_prediction_forest_poisons_rows():
    c, plan = _plan(random_forest_pmml(n_trees=16, depth=5, n_features=8, n_classes=3, seed=5,
                                       missing_strategy="nullPrediction"))
    assert plan.blob_nan is None and not plan.variant & VAR_NAN_FAST  # per-node missing test
    X = stream_matrix(3000, 8, seed=6, missing_rate=0.03)
    _, vref = c.score_matrix_oracle(X)
    assert 0 < vref.sum() < len(X)
    _check(c, plan, X)


@pytest.mark.parametrize("F,rows", [(100, 128), (200, 64)])
def test_wide_records_row_tiles_and_compaction(F, rows):
    """> 64 staged columns: smaller row tiles keep the planes in LDS; the trees of a sparse
    model read few of many columns and only those are staged."""
    c, plan = _plan(gbdt_pmml(n_trees=30, depth=6, n_features=F, seed=F))
    assert plan.variant & 3 == 1
    n_used = len({int(f) for t in plan.spec.trees for f in t.feature if f >= 0})
    assert plan.n_stage == n_used
    assert plan.rows_wide == next(r for r, lim in ((256, 64), (128, 128), (64, 256)) if n_used <= lim)
    if n_used > 128:
        assert rows == 64 and plan.rows_wide == 64
    X = stream_matrix(700, F, seed=1, missing_rate=0.05)
    _check(c, plan, X, tol=1e-4)


def test_feature_compaction_map():
    c, plan = _plan(gbdt_pmml(n_trees=3, depth=2, n_features=300, seed=7))
    assert plan.feat_map is not None and plan.n_stage <= 12 and plan.rows_wide == 256
    _check(c, plan, stream_matrix(600, 300, seed=8, missing_rate=0.1), tol=1e-4)


@pytest.mark.parametrize("case", ["general-reg", "general-cls", "vote8", "slot", "pointer", "fp8"])
def test_plan_state_roundtrip_dry(case):
    """Every TreePlan variant exports / re-imports its state (the RCCL model replication path)."""
    import sys

    from flink_jpmml_amd.runtime.plans import DevicePlan

    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_general_tree import general_tree_doc

    txt, kw = {
        "general-reg": (general_tree_doc(4, "defaultChild", "returnLastPrediction", n_trees=5), {}),
        "general-cls": (general_tree_doc(4, "defaultChild", "returnLastPrediction", n_trees=5,
                                         classification=True), {}),
        "vote8": (random_forest_pmml(n_trees=8, depth=4, n_features=6, n_classes=3), {}),
        "slot": (gbdt_pmml(n_trees=4, depth=3, n_features=6, objective="multiclass", n_classes=3), {}),
        "pointer": (gbdt_pmml(n_trees=4, depth=3, n_features=6), {"layout": "pointer"}),
        "fp8": (gbdt_pmml(n_trees=4, depth=3, n_features=6), {"precision": "fp8"}),
    }[case]
    c, plan = _plan(txt, **kw)
    with lowering_dry_run():
        meta, tensors = plan.export_state()
        q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, torch.device("cpu"))
    for k in TreePlan._STATE:
        a, b = getattr(plan, k), getattr(q, k)
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b), k
        else:
            assert a == b, k


def test_many_class_chain_general_slots_with_intercept_stumps():
    """K > 8 classes: the narrow kernel's LDS class slots; intercepts travel as constant stump
    trees (to_general) and must be counted in n_trees."""
    from flink_jpmml_amd.runtime.plans import TB

    c, p = _plan(gbdt_pmml(n_trees=10, depth=4, n_features=12, objective="multiclass", n_classes=12, seed=2))
    assert p.variant == 0 and p.general == 1 and p.C == 12 and p.n_trees == 120 + 11
    X = stream_matrix(2000, 12, seed=3)
    ref, _ = c.score_matrix_oracle(X)
    D = p.depth
    NI, NL = (1 << D) - 1, 1 << D
    blob = p.blob.numpy().view(np.uint32).reshape(p.n_trees, p.rec_words)
    slots = p.slots.numpy()
    acc = np.zeros((len(X), p.C))
    Xf = X.astype(np.float32)
    for t in range(p.n_trees):
        T = blob[t, 0:2 * NI:2].view(np.float32)
        meta = blob[t, 1:2 * NI:2]
        leaves = blob[t, 2 * NI:2 * NI + NL].view(np.float32)
        j = np.ones(len(X), np.int64)
        for _ in range(D):
            j = 2 * j + (Xf[np.arange(len(X)), meta[j - 1] // (TB * 4)] >= T[j - 1])
        acc[:, slots[t]] += leaves[j - NL]
    tab = np.array([float(v) for v in p.labels])
    assert (tab[np.argmax(acc, axis=1)] == ref).all()


@pytest.mark.parametrize("missing", [0.0, 0.04])
def test_monotone_derived_fields_fold_into_thresholds(missing):
    """StandardScaler / NormContinuous / decreasing affine derived fields read only as split
    fields: folded into fp32 thresholds on the raw inputs (no derive pass), exact vs the oracle."""
    from flink_jpmml_amd.runtime.derive import plan_field_layout
    from flink_jpmml_amd.runtime.plans import compile_plan

    txt = gbdt_pmml(n_trees=40, depth=6, n_features=12, scaled=True, seed=11)
    c = CompiledPmml.from_string(txt)
    layout = plan_field_layout(c, allow_fold=True)
    assert layout.program is None and len(layout.folds) == 12
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert type(plan).__name__ == "TreePlan" and plan.variant & 3 == 1
    _check(c, plan, stream_matrix(6000, 12, seed=5, missing_rate=missing), tol=1e-4)


def test_fold_splits_exact_on_the_fp32_line():
    from flink_jpmml_amd.models.tree import OP_GE, OP_GT, OP_LE, OP_LT
    from flink_jpmml_amd.runtime.derive import fold_splits

    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.standard_normal(200_000), np.linspace(-3, 3, 200_001)]).astype(np.float32)
    xs = xs.astype(np.float64)
    for f in (lambda x: (x - 0.3) / 1.25, lambda x: (0.5 - x) * 0.8, lambda x: np.clip(x, -1, 1)):
        ts = np.array([-2.0, -0.7, 0.0, 0.123456789, 0.9, 5.0])
        for op in (OP_LT, OP_LE, OP_GT, OP_GE):
            ops = np.full(len(ts), op, np.int8)
            o2, t2 = fold_splits(f, ops, ts)
            for i, t in enumerate(ts):
                y = f(xs)
                P = {OP_LT: y < t, OP_LE: y <= t, OP_GT: y > t, OP_GE: y >= t}[op]
                Q = xs < t2[i] if o2[i] == OP_LT else xs >= t2[i]
                assert (P == Q).all(), (op, t)


def test_fold_skips_derived_fields_with_mining_treatment():
    """A segment MiningField that treats the derived value itself (here: missing replacement) is
    applied to d, not x — such a field must not be folded (derive pass instead)."""
    from flink_jpmml_amd.runtime.derive import plan_field_layout

    txt = gbdt_pmml(n_trees=3, depth=3, n_features=4, scaled=True, seed=2)
    i = txt.index('<MiningField name="f0"/>', txt.index('<Segment'))  # the first segment's schema
    txt = txt[:i] + '<MiningField name="d(f1)" missingValueReplacement="0.5"/>' + txt[i:]
    c = CompiledPmml.from_string(txt)
    layout = plan_field_layout(c, allow_fold=True)
    assert layout.folds is None and layout.program is not None
