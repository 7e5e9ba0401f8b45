"""CPU checks of the device lowering: a numpy emulation of the PERFECT-layout traversal kernel
(heap index, canonical ``x >= T`` splits, default-right bit words, fused epilogue) must agree with
the float64 oracle — this pins the packing format without a GPU."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.models.tree import OP_GE, OP_GT, OP_LE, OP_LT
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import TB, _nan_planes, _perfect_pack, _pointer_pack, canonical_threshold, ensemble_spec, to_general


def emulate_perfect(c, X):
    spec = to_general(ensemble_spec(c))  # the narrow kernel's P = C payload form
    D = max(t.depth for t in spec.trees)
    P = spec.P
    blob, rec, _ = _perfect_pack(spec.trees, spec.weights, P, D)
    assert rec % 4 == 0
    NI, NL = (1 << D) - 1, 1 << D
    Xf = X.astype(np.float32)
    n = len(X)
    acc = np.zeros((n, P), np.float32)
    for ti in range(blob.shape[0]):
        T = blob[ti, 0:2 * NI:2].view(np.float32)
        meta = blob[ti, 1:2 * NI:2]
        leaves = blob[ti, 2 * NI:2 * NI + NL * P].view(np.float32).reshape(NL, P)
        drw = blob[ti, 2 * NI + NL * P: 2 * NI + NL * P + (NI + 31) // 32]
        j = np.ones(n, np.int64)
        pz = np.zeros(n, dtype=bool)
        for _ in range(D):
            f = meta[j - 1] // (TB * 4)
            x = Xf[np.arange(n), f]
            dr = (drw[(j - 1) >> 5] >> ((j - 1) & 31)) & 1
            right = (x >= T[j - 1]) | (np.isnan(x) & (dr == 1))
            pz |= np.isnan(x)
            j = 2 * j + right
        null_tree = (drw[NI >> 5] >> (NI & 31)) & 1  # tree-level null-on-missing flag
        acc += np.where((pz & (null_tree == 1))[:, None], np.float32(np.nan), leaves[j - NL])
    return spec, acc


def emulate_pointer(c, X):
    spec = to_general(ensemble_spec(c))
    nodes, leaves, roots, _ = _pointer_pack(spec.trees, spec.weights, spec.P)
    Xf = X.astype(np.float32)
    acc = np.zeros((len(X), spec.P), np.float32)
    for r in range(len(X)):
        for root in roots:
            code = int(root)
            while code >= 0:
                T, meta, lc, rc = nodes[code]
                f = int(meta) & 0xFFFF
                f = f // (TB * 4)
                x = Xf[r, f]
                right = (x >= np.uint32(T).view(np.float32)) or (np.isnan(x) and (int(meta) >> 31) & 1)
                code = int(np.int32(np.uint32(rc if right else lc)))
            acc[r] += leaves[~code]
    return spec, acc


def _scores(spec, acc):
    """Epilogue emulation; rows whose accumulator is NaN (a null tree) score NaN (EmptyScore)."""
    e = spec.epi
    bad = np.isnan(acc).any(axis=1)
    if e["mode"] == 0:
        return np.where(bad, np.nan, e["a"] * acc[:, 0] + e["b"])
    tab = np.array([float(x) for x in spec.labels])
    if e["mode"] == 1:
        p0 = 1.0 / (1.0 + np.exp(-(e["a"] * acc[:, 0] + e["b"])))
        return np.where(bad, np.nan, tab[np.where(p0 >= 0.5, 0, 1)])
    return np.where(bad, np.nan, tab[np.argmax(np.nan_to_num(acc), axis=1)])


@pytest.mark.parametrize("kind", ["regression", "binary", "rf"])
def test_perfect_layout_emulation_matches_oracle(kind):
    if kind == "rf":
        txt = random_forest_pmml(n_trees=15, depth=6, n_features=10, n_classes=3, seed=3)
    else:
        txt = gbdt_pmml(n_trees=40, depth=5, n_features=12, seed=1, objective=kind)
    c = CompiledPmml.from_string(txt)
    X = stream_matrix(3000, c.n_features, seed=2, missing_rate=0.05)
    ref, vref = c.score_matrix_oracle(X)
    spec, acc = emulate_perfect(c, X)
    out = _scores(spec, acc)
    assert vref.all()
    if kind == "regression":
        assert np.max(np.abs(out - ref)) < 1e-5
    else:
        assert (out == ref).all()


def emulate_perfect_fast(c, X, nan_planes=False):
    """Byte-address form used by the wide kernel's fast path (tree.hip::traverse_fast_g): node
    address u' = 2u + (8 - b0) + 8r, leaf pair at u + 8 + 8*NI - 4*NL on the last level.
    ``nan_planes``: default-right nodes read the second (NaN -> +inf) feature plane."""
    spec = ensemble_spec(c)
    D = max(t.depth for t in spec.trees)
    blob, rec, _ = _perfect_pack(spec.trees, spec.weights, 1, D)
    if nan_planes:
        blob = _nan_planes(blob, D, X.shape[1])
        X = np.concatenate([X, np.where(np.isnan(X), np.inf, X)], axis=1)
    mem = blob.reshape(-1)
    NI, NL = (1 << D) - 1, 1 << D
    C = 8 + 8 * NI - 4 * NL
    Xf = X.astype(np.float32)
    rows = np.arange(len(X))
    acc = np.zeros(len(X), np.float32)
    for t in range(blob.shape[0]):
        b0 = t * rec * 4
        u = np.full(len(X), b0, np.int64)
        for _ in range(D - 1):
            x = Xf[rows, mem[u // 4 + 1] // (TB * 4)]
            u = 2 * u + (8 - b0) + 8 * (x >= mem[u // 4].view(np.float32))
        x = Xf[rows, mem[u // 4 + 1] // (TB * 4)]
        right = x >= mem[u // 4].view(np.float32)
        acc += np.where(right, mem[(u + C) // 4 + 1].view(np.float32), mem[(u + C) // 4].view(np.float32))
    return acc


@pytest.mark.parametrize("depth", [1, 3, 6])
def test_wide_fast_path_addressing(depth):
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=12, depth=depth, n_features=7, seed=depth))
    X = stream_matrix(257, 7, seed=1)
    _, ref = emulate_perfect(c, X)
    np.testing.assert_array_equal(emulate_perfect_fast(c, X), ref[:, 0])


@pytest.mark.parametrize("depth", [2, 6])
def test_nan_planes_fast_path_matches_missing_path(depth):
    """Missing values on the fast path: the default direction is encoded in the feature plane."""
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=20, depth=depth, n_features=9, seed=depth + 10))
    X = stream_matrix(500, 9, seed=3, missing_rate=0.2)
    _, ref = emulate_perfect(c, X)
    np.testing.assert_array_equal(emulate_perfect_fast(c, X, nan_planes=True), ref[:, 0])
    assert not np.array_equal(emulate_perfect_fast(c, X), ref[:, 0])  # without the planes: wrong


def test_pointer_layout_emulation_matches_oracle():
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=6, depth=7, n_features=9, seed=4))
    X = stream_matrix(200, 9, seed=5, missing_rate=0.1)
    ref, _ = c.score_matrix_oracle(X)
    spec, acc = emulate_pointer(c, X)
    assert np.max(np.abs(_scores(spec, acc) - ref)) < 1e-5


@pytest.mark.parametrize("op", [OP_LT, OP_LE, OP_GT, OP_GE])
def test_canonical_threshold_exact_for_fp32_inputs(op):
    """For every fp32 x near t the canonical `x >= T` test reproduces the fp64 comparison."""
    rng = np.random.default_rng(op)
    for t in list(rng.standard_normal(200)) + [0.1, 0.5, 1e-30, -2.5, 3.0, 16777217.0]:
        T, swap = canonical_threshold(op, float(t))
        f = np.float32(t)
        cands = [f, np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf)),
                 np.nextafter(np.nextafter(f, np.float32(np.inf)), np.float32(np.inf))]
        for x in cands:
            xd = float(x)
            first = {OP_LT: xd < t, OP_LE: xd <= t, OP_GT: xd > t, OP_GE: xd >= t}[op]
            right = bool(np.float32(x) >= np.float32(T))
            assert first == (right if swap else not right), (op, t, x, T)


# ---------------------------------------------------------------------------- MLP fragment packing
def _acc_row(r, h):
    return (r & 3) + 8 * (r >> 2) + 4 * h


def emulate_mlp_wave(layers, X32, precision):
    """Emulate csrc/mlp.hip for one wave (32 rows) at the MFMA fragment level: A fragments from
    pack_mlp_weights, B fragments from staged inputs (layer 0) or from the previous layer's
    accumulator registers (layers >= 1), C/D register layout of the 32x32 tile."""
    from flink_jpmml_amd.models.neural import activate
    from flink_jpmml_amd.runtime.nn_plans import pack_mlp_weights

    w, bias, meta = pack_mlp_weights([(W, b) for W, b, _ in layers], precision)
    bf16 = precision == "bf16"
    kstep = 16 if bf16 else 2
    lane = np.arange(64)
    hh, col = lane >> 5, lane & 31
    regs_prev = None  # [tiles][64 lanes][16 regs]
    for L, ((kp, mp, mreal, wo, bo), (_, _, act)) in enumerate(zip(meta, layers)):
        mtiles, ksteps = mp // 32, kp // kstep
        nfr = 8 if bf16 else 1
        frags = w[wo: wo + mtiles * ksteps * 64 * nfr].reshape(mtiles, ksteps, 64, nfr)
        D = np.zeros((mtiles, 32, 32))
        for t in range(mtiles):
            D[t] = bias[bo + 32 * t: bo + 32 * t + 32][:, None]
        for s in range(ksteps):
            Bl = np.zeros((kstep, 32))
            for l in range(64):
                for j in range(nfr):
                    k = (8 * hh[l] + j) if bf16 else hh[l]
                    if L == 0:
                        feat = (16 * s + 8 * hh[l] + j) if bf16 else (2 * s + hh[l])
                        Bl[k, col[l]] = X32[col[l], feat] if feat < X32.shape[1] else 0.0
                    elif bf16:
                        tp, sp = s // 2, s % 2
                        Bl[k, col[l]] = regs_prev[tp][l][8 * sp + j]
                    else:
                        tp, r = s // 16, s % 16
                        Bl[k, col[l]] = regs_prev[tp][l][r]
            for t in range(mtiles):
                Al = np.zeros((32, kstep))
                for l in range(64):
                    for j in range(nfr):
                        k = (8 * hh[l] + j) if bf16 else hh[l]
                        Al[col[l], k] = frags[t, s, l, j]
                D[t] += Al @ Bl
        D = activate(act, D)
        regs_prev = [[[D[t][_acc_row(r, hh[l]), col[l]] for r in range(16)] for l in range(64)]
                     for t in range(mtiles)]
    return D[0]  # [units (tile 0), 32 rows]


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_mlp_fragment_packing_matches_dense_forward(precision):
    rng = np.random.default_rng(0)
    dims = [(20, 40), (40, 33), (33, 3)]  # odd sizes exercise K and M padding
    layers = [(rng.standard_normal(d), rng.standard_normal(d[1]), a)
              for d, a in zip(dims, ["rectifier", "tanh", "identity"])]
    X = rng.standard_normal((32, 20))
    from flink_jpmml_amd.models.neural import activate

    H = X
    for W, b, act in layers:
        H = activate(act, H @ W + b)
    out = emulate_mlp_wave(layers, X, precision)
    assert np.allclose(out[:3].T, H, atol=1e-9)


@pytest.mark.parametrize("kind", ["regression", "rf"])
def test_null_prediction_trees_poison_rows(kind):
    """sklearn-style ``nullPrediction`` trees: a missing value at a visited split voids the tree,
    and with it the ensemble's prediction (MiningModel ``continue`` rule) -> EmptyScore."""
    if kind == "rf":
        txt = random_forest_pmml(n_trees=12, depth=5, n_features=8, n_classes=3, seed=4,
                                 missing_strategy="nullPrediction")
    else:
        txt = gbdt_pmml(n_trees=25, depth=4, n_features=8, seed=3, missing_strategy="nullPrediction")
    c = CompiledPmml.from_string(txt)
    assert all(t.null_missing for t in ensemble_spec(c).trees)
    X = stream_matrix(3000, 8, seed=6, missing_rate=0.03)
    ref, vref = c.score_matrix_oracle(X)
    assert 0 < vref.sum() < len(X)  # both outcomes occur
    spec, acc = emulate_perfect(c, X)
    out = _scores(spec, acc)
    assert (np.isfinite(out) == vref).all()
    if kind == "rf":
        assert (out[vref] == ref[vref]).all()
    else:
        assert np.max(np.abs(out[vref] - ref[vref])) < 1e-5
    # pointer layout: per-node null bit (meta bit 30)
    nodes, _, _, _ = _pointer_pack(spec.trees, spec.weights, spec.P)
    internal = nodes[:, 2].astype(np.int64) != nodes[:, 3].astype(np.int64)
    assert ((nodes[internal, 1] >> 30) & 1).all()


def emulate_leaf8(c, X):
    """fp8-leaf wide-kernel format: the e4m3 leaf pair sits in bits [31:16] of each last-level
    node's meta; the feature offset is the low half."""
    from flink_jpmml_amd.runtime.plans import _leaf8_pack, dequantize_fp8

    spec = ensemble_spec(c)
    D = max(t.depth for t in spec.trees)
    blob, _, _ = _perfect_pack(spec.trees, spec.weights, 1, D)
    blob8, rec8, scale = _leaf8_pack(blob, D)
    NI = (1 << D) - 1
    assert rec8 == ((2 * NI + (NI + 31) // 32 + 3) & ~3) and rec8 % 4 == 0
    Xf = X.astype(np.float32)
    rows = np.arange(len(X))
    acc = np.zeros(len(X), np.float32)
    for t in range(blob8.shape[0]):
        T = blob8[t, 0:2 * NI:2].view(np.float32)
        meta = blob8[t, 1:2 * NI:2]
        j = np.ones(len(X), np.int64)
        for d in range(D):
            m = meta[j - 1]
            x = Xf[rows, (m & 0xFFFF) // (TB * 4)]
            right = x >= T[j - 1]
            if d == D - 1:
                byte = np.where(right, m >> 24, (m >> 16) & 0xFF).astype(np.uint8)
                acc += dequantize_fp8(byte)
            else:
                j = 2 * j + right
    return spec, acc * np.float32(scale), blob


@pytest.mark.parametrize("depth", [1, 4, 6])
def test_fp8_leaf_packing(depth):
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=60, depth=depth, n_features=9, seed=depth, objective="binary"))
    X = stream_matrix(2000, 9, seed=2)
    spec, acc8, _ = emulate_leaf8(c, X)
    _, acc32 = emulate_perfect(c, X)
    # decisions are fp32-exact; only leaf values are quantised (e4m3: 3 mantissa bits, |rel err| <= 1/16)
    leaf_max = max(float(np.max(np.abs(t.leaf_value[t.feature < 0]))) for t in spec.trees)
    assert np.max(np.abs(acc8 - acc32[:, 0])) <= 60 * leaf_max / 16 + 1e-6
    ref, _ = c.score_matrix_oracle(X)
    agree = (_scores(spec, acc8[:, None]) == ref).mean()
    assert agree > 0.97


def test_vectorised_perfect_pack_is_bit_identical():
    """The level-at-a-time packer (model load time) == the per-node reference, for regression /
    K-class / vote8 / null-prediction / sparse trees, both strides, with a column map, and P > 1."""
    import numpy as np

    from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import TB, _perfect_pack_loop, _perfect_pack_vec, ensemble_spec, to_general

    cases = [(gbdt_pmml(n_trees=30, depth=6, n_features=32, seed=1), None, False),
             (gbdt_pmml(n_trees=10, depth=5, n_features=10, objective="multiclass", n_classes=4, seed=2), None, False),
             (random_forest_pmml(n_trees=20, depth=7, n_features=12, n_classes=3, seed=3), "vote8", False),
             (random_forest_pmml(n_trees=20, depth=5, n_features=12, n_classes=3, seed=4,
                                 missing_strategy="nullPrediction"), None, False),
             (random_forest_pmml(n_trees=20, depth=5, n_features=12, n_classes=3, seed=6), None, True),
             (gbdt_pmml(n_trees=30, depth=6, n_features=20, seed=5, p_split=0.6), None, False)]
    for txt, leaf_bits, general in cases:
        spec = ensemble_spec(CompiledPmml.from_string(txt))
        if general:
            spec = to_general(spec)
        D = max(t.depth for t in spec.trees)
        NI, NL = (1 << D) - 1, 1 << D
        rec = ((2 * NI + NL * spec.P + (NI + 31) // 32) + 3) & ~3
        for stride, fmap in ((TB, None), (256, {f: (f * 7) % 40 for f in range(40)})):
            a = _perfect_pack_loop(spec.trees, spec.weights, spec.P, D, stride, fmap, leaf_bits, rec)
            b = _perfect_pack_vec(spec.trees, spec.weights, spec.P, D, stride, fmap, leaf_bits, rec)
            assert np.array_equal(a[0], b[0]) and a[1:] == b[1:], (leaf_bits, general, stride)


def test_null_prediction_padding_reads_a_visited_column():
    """An unbalanced nullPrediction tree: a leaf above the PERFECT depth is padded down to depth D,
    and the padded nodes must read a column the walk already visited (their parent split's), not
    column 0 — a row whose path never touches the missing column 0 keeps its prediction (the
    r5av chain-fuzz failure: 1-2.5 % of rows wrongly EmptyScore on the device)."""
    ns = "http://www.dmg.org/PMML-4_4"
    doc = (f'<PMML version="4.4" xmlns="{ns}"><DataDictionary>'
           '<DataField name="f0" optype="continuous" dataType="double"/>'
           '<DataField name="f1" optype="continuous" dataType="double"/>'
           '<DataField name="y" optype="continuous" dataType="double"/></DataDictionary>'
           '<TreeModel functionName="regression" missingValueStrategy="nullPrediction" splitCharacteristic="binarySplit">'
           '<MiningSchema><MiningField name="y" usageType="target"/><MiningField name="f0"/><MiningField name="f1"/>'
           '</MiningSchema><Node id="r" score="0"><True/>'
           '<Node id="a" score="1.5"><SimplePredicate field="f1" operator="lessThan" value="0.2"/></Node>'
           '<Node id="b" score="2"><SimplePredicate field="f1" operator="greaterOrEqual" value="0.2"/>'
           '<Node id="c" score="-1"><SimplePredicate field="f0" operator="lessThan" value="0"/></Node>'
           '<Node id="d" score="4"><SimplePredicate field="f0" operator="greaterOrEqual" value="0"/></Node>'
           '</Node></Node></TreeModel></PMML>')
    c = CompiledPmml.from_string(doc)
    X = np.array([[np.nan, -1.0], [np.nan, 1.0], [0.5, np.nan], [-0.5, 1.0], [np.nan, 0.1]])
    ref, vref = c.score_matrix_oracle(X)
    assert list(vref) == [True, False, False, True, True]
    spec, acc = emulate_perfect(c, X)
    out = _scores(spec, acc)
    assert (np.isfinite(out) == vref).all()
    assert np.allclose(out[vref], ref[vref])
