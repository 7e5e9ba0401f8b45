"""Native host tree walk (``native/csrc/tree_walk.cpp``, ``models/native_tree.py``) vs the numpy
walk it replaces (the host scoring path).

The native walker must choose the numpy walk's node on every row — same float64 comparisons over
the same prepared columns, same three-valued predicate logic, same missing-value and no-true-child
strategies — and the native ensemble sum must be bit-identical to ``_regress``'s ``np.sum``.
Checked on seeded random TreeModels (1-4 children per node, Simple / SimpleSet / Compound
(and/or/xor/surrogate) / isMissing / True / False predicates, every ``missingValueStrategy`` x
``noTrueChildStrategy``, defaultChild attributes that name a child or not, missing inputs, values
on the split points), on binary GBDT ensembles (the fixed-depth and perfect walks, AVX-512 and
scalar), and on the reference fixtures."""

from __future__ import annotations

import os
import random

import numpy as np
import pytest

from flink_jpmml_amd.models.native_tree import native_available
from flink_jpmml_amd.runtime.compiled import CompiledPmml

pytestmark = pytest.mark.skipif(not native_available(), reason="native fast path not built")

NF = 4
VALUES = [-1.0, -0.5, 0.0, 0.25, 0.5, 1.0]
STRATS = ["none", "lastPrediction", "nullPrediction", "defaultChild", "weightedConfidence", "aggregateNodes"]


def _pred(rng: random.Random, depth: int) -> str:
    if depth == 0 or rng.random() < 0.75:
        k = rng.randrange(10)
        f = f"f{rng.randrange(NF)}"
        if k == 0:
            return "<True/>"
        if k == 1:
            return "<False/>"
        if k == 2:
            return f'<SimplePredicate field="{f}" operator="{rng.choice(["isMissing", "isNotMissing"])}"/>'
        if k == 3:
            vals = " ".join(repr(v) for v in rng.sample(VALUES, rng.randrange(1, 4)))
            op = rng.choice(["isIn", "isNotIn"])
            return f'<SimpleSetPredicate field="{f}" booleanOperator="{op}"><Array type="real">{vals}</Array>' \
                   "</SimpleSetPredicate>"
        op = rng.choice(["equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual"])
        return f'<SimplePredicate field="{f}" operator="{op}" value="{rng.choice(VALUES)!r}"/>'
    op = rng.choice(["and", "or", "xor", "surrogate"])
    return f'<CompoundPredicate booleanOperator="{op}">' + "".join(
        _pred(rng, depth - 1) for _ in range(rng.randrange(2, 4))) + "</CompoundPredicate>"


def _node(rng: random.Random, depth: int, ids: list, classification: bool, pred: str,
          consistent: bool = False) -> str:
    """``consistent``: a classification node's score is its distribution's first argmax (what
    exporters write; the device label is the argmax of the class probabilities)."""
    nid = f"n{len(ids)}"
    ids.append(nid)
    cats = ["a", "b", "c"]
    score = rng.choice(cats) if classification else repr(round(rng.uniform(-3, 3), 3))
    dist = ""
    if classification:
        cnts = [rng.randrange(1, 9) for _ in cats]
        if consistent:
            score = cats[int(np.argmax(cnts))]
        dist = "".join(f'<ScoreDistribution value="{c}" recordCount="{n}"/>' for c, n in zip(cats, cnts))
    rc = f' recordCount="{rng.randrange(1, 50)}"'
    if depth == 0 or rng.random() < 0.2:
        return f'<Node id="{nid}" score="{score}"{rc}>{pred}{dist}</Node>'
    nch = rng.choice([1, 2, 2, 2, 3, 4])
    kids = []
    if nch == 2 and rng.random() < 0.5:  # the exporters' binary split (FAST nodes)
        f = f"f{rng.randrange(NF)}"
        op = rng.choice(["lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual"])
        v = rng.choice(VALUES)
        neg = {"lessThan": "greaterOrEqual", "lessOrEqual": "greaterThan", "greaterThan": "lessOrEqual",
               "greaterOrEqual": "lessThan"}[op]
        second = "<True/>" if rng.random() < 0.5 else f'<SimplePredicate field="{f}" operator="{neg}" value="{v!r}"/>'
        preds = [f'<SimplePredicate field="{f}" operator="{op}" value="{v!r}"/>', second]
    else:
        preds = [_pred(rng, 2) for _ in range(nch)]
    first_kid = len(ids)
    for p in preds:
        kids.append(_node(rng, depth - 1, ids, classification, p, consistent))
    dflt = ""
    if rng.random() < 0.8:
        dflt = f' defaultChild="{ids[first_kid] if rng.random() < 0.6 else ids[-1]}"'
    return f'<Node id="{nid}" score="{score}"{rc}{dflt}>{pred}{dist}{"".join(kids)}</Node>'


def _header(target_xml: str) -> str:
    fields = "".join(f'<DataField name="f{j}" optype="continuous" dataType="double"/>' for j in range(NF))
    return ('<PMML xmlns="http://www.dmg.org/PMML-4_4" version="4.4"><Header/><DataDictionary>'
            f'{fields}{target_xml}</DataDictionary>')


def _ms() -> str:
    return '<MiningSchema><MiningField name="y" usageType="target"/>' + \
        "".join(f'<MiningField name="f{j}"/>' for j in range(NF)) + "</MiningSchema>"


def random_tree_doc(seed: int) -> str:
    rng = random.Random(seed)
    strat = STRATS[seed % len(STRATS)]
    classification = strat in ("weightedConfidence", "aggregateNodes") or rng.random() < 0.3
    notrue = rng.choice(["returnNullPrediction", "returnLastPrediction"])
    root = _node(rng, rng.randrange(2, 6), [], classification, "<True/>" if rng.random() < 0.85 else _pred(rng, 1))
    tgt = ('<DataField name="y" optype="categorical" dataType="string"><Value value="a"/><Value value="b"/>'
           '<Value value="c"/></DataField>') if classification else \
        '<DataField name="y" optype="continuous" dataType="double"/>'
    fn = "classification" if classification else "regression"
    return (_header(tgt) + f'<TreeModel functionName="{fn}" missingValueStrategy="{strat}" '
            f'noTrueChildStrategy="{notrue}">{_ms()}{root}</TreeModel></PMML>')


def _inputs(seed: int, n: int = 3000) -> np.ndarray:
    rng = np.random.default_rng(seed)
    X = rng.choice(np.array(VALUES + [0.1, -0.7, 2.0]), size=(n, NF))
    X[rng.random((n, NF)) < 0.15] = np.nan
    return X


def _numpy_only(c: CompiledPmml) -> None:
    """Force the numpy walk on every evaluator of ``c`` (the semantic reference)."""
    stack = [c.evaluator]
    while stack:
        ev = stack.pop()
        ev._native = None
        stack.extend(getattr(ev, "sub", []) or [])


@pytest.mark.parametrize("seed", range(60))
def test_random_tree_leaves_match_numpy_walk(seed):
    doc = random_tree_doc(seed)
    c = CompiledPmml.from_string(doc)
    ev = c.evaluator
    X = _inputs(seed)
    P, _ = c.prepare(X)
    cols = c.columns(P)
    prog = ev.native_program()
    assert prog is not None, "every generated tree is natively encodable"
    got = ev.leaf_index(c.columns(P))
    want = ev.leaf_index_numpy(cols)
    np.testing.assert_array_equal(got, want)
    # and the whole oracle (classification mixtures, targets) agrees
    s1, v1 = c.score_matrix_oracle(X)
    c2 = CompiledPmml.from_string(doc)
    _numpy_only(c2)
    s2, v2 = c2.score_matrix_oracle(X)
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(s1[v1], s2[v2])


def _gbdt_doc(seed: int, method: str = "sum", n_trees: int = 37) -> str:
    from flink_jpmml_amd.bench import synth

    doc = synth.gbdt_pmml(n_trees=n_trees, depth=3 + seed % 5, n_features=8, seed=seed)
    if method != "sum":
        doc = doc.replace('multipleModelMethod="sum"', f'multipleModelMethod="{method}"')
    return doc


@pytest.mark.parametrize("method", ["sum", "average", "weightedSum", "weightedAverage", "median", "max"])
@pytest.mark.parametrize("seed", [0, 3, 7])
def test_forest_aggregate_is_bit_identical_to_numpy(method, seed):
    from flink_jpmml_amd.bench import synth

    doc = _gbdt_doc(seed, method)
    assert f'multipleModelMethod="{method}"' in doc
    X = synth.stream_matrix(2000, 8, seed=seed + 1, missing_rate=0.05)
    X[:50] = np.round(X[:50], 1)  # values on / next to the split points
    c = CompiledPmml.from_string(doc)
    assert c.evaluator.native_forest() is not None
    s1, v1 = c.score_matrix_oracle(X)
    c2 = CompiledPmml.from_string(doc)
    _numpy_only(c2)
    s2, v2 = c2.score_matrix_oracle(X)
    np.testing.assert_array_equal(v1, v2)
    assert np.array_equal(s1[v1], s2[v2])  # bit-identical, not approximately equal


@pytest.mark.parametrize("seed", [0, 2, 4])  # depths 3, 5, 7: register levels (<= 32 nodes) and gathers
def test_scalar_and_avx512_walks_agree(monkeypatch, seed):
    from flink_jpmml_amd.bench import synth

    c = CompiledPmml.from_string(_gbdt_doc(seed, n_trees=64))
    prog = c.evaluator.native_forest()
    X = np.ascontiguousarray(synth.stream_matrix(3001, 8, seed=9, missing_rate=0.1))
    fast = prog.leaves(X)
    monkeypatch.setenv("FJA_WALK_SCALAR", "1")
    slow = prog.leaves(X)
    np.testing.assert_array_equal(fast, slow)
    # and the general (non-fixed) walk on a single row agrees too: rows are walked one by one
    # whenever a block is shorter than the interleave width
    one = prog.leaves(np.ascontiguousarray(X[:7]))
    np.testing.assert_array_equal(one, fast[:, :7])
    monkeypatch.delenv("FJA_WALK_SCALAR")
    # single records on the AVX-512 path: 8 trees per vector instead of 32 rows
    for i in (0, 5, 17):
        np.testing.assert_array_equal(prog.leaves(np.ascontiguousarray(X[i:i + 1])), fast[:, i:i + 1])


def test_pairwise_sum_matches_numpy_for_every_width():
    """The native row sum reproduces np.sum(axis=1) of a C-contiguous matrix for any tree count."""
    from flink_jpmml_amd.models.native_tree import ForestProgram

    for n_trees in (1, 2, 7, 8, 9, 127, 128, 129, 257, 1000):
        doc = _gbdt_doc(1, n_trees=n_trees)
        c = CompiledPmml.from_string(doc)
        prog = c.evaluator.native_forest()
        assert isinstance(prog, ForestProgram) and prog.n_trees == n_trees
        X = np.random.default_rng(n_trees).normal(size=(300, len(prog.fields)))
        V = prog.values(X)
        np.testing.assert_array_equal(prog.sums(X), np.sum(V, axis=1))
        w = np.random.default_rng(1).uniform(0.1, 2, n_trees)
        np.testing.assert_array_equal(prog.sums(X, w), np.sum(V * w[None, :], axis=1))


def test_malformed_program_raises_instead_of_reading_out_of_bounds():
    from flink_jpmml_amd.native import fastpath

    c = CompiledPmml.from_string(_gbdt_doc(2, n_trees=3))
    prog = c.evaluator.native_forest()
    ni, nd, kids, pi, pd, ai, ad, roots, modes, lv = prog.arrays()
    X = np.zeros((4, len(prog.fields)))
    out = np.empty((3, 4), dtype=np.int32)
    bad = ni.copy()
    bad[8 * 0 + 5] = 10 ** 6  # a FAST child pointing past the node table
    with pytest.raises(ValueError):
        fastpath().forest_leaves(bad, nd, kids, pi, pd, ai, ad, roots, modes, X, X.shape[1], out)
    with pytest.raises(ValueError):
        fastpath().forest_leaves(ni, nd, kids, pi, pd, ai, ad, roots + 10 ** 6, modes, X, X.shape[1], out)
    with pytest.raises(ValueError):  # X narrower than the fields the program reads
        fastpath().forest_leaves(ni, nd, kids, pi, pd, ai, ad, roots, modes, np.zeros((4, 1)), 1, out)


def test_reference_fixtures_score_like_the_numpy_walk(fixtures_dir):
    for name, path in sorted(fixtures_dir.items()):
        if not str(path).endswith(".pmml") and not str(path).endswith(".xml"):
            continue
        try:
            c = CompiledPmml.load(path)
        except Exception:  # noqa: BLE001 - deliberately broken fixtures
            continue
        if not c.active_fields:
            continue
        X = np.random.default_rng(0).uniform(0.0, 8.0, size=(500, c.n_features))
        X[::7, 0] = np.nan
        s1, v1 = c.score_matrix_oracle(X)
        c2 = CompiledPmml.load(path)
        _numpy_only(c2)
        s2, v2 = c2.score_matrix_oracle(X)
        np.testing.assert_array_equal(v1, v2, err_msg=name)
        np.testing.assert_array_equal(s1[v1], s2[v2], err_msg=name)


@pytest.mark.skipif(os.environ.get("FJA_PERF_TESTS") != "1", reason="timing check (FJA_PERF_TESTS=1)")
def test_host_gbdt_throughput():
    import time

    from flink_jpmml_amd.bench import synth

    c = CompiledPmml.from_string(synth.gbdt_pmml(n_trees=1000, depth=6, n_features=32, seed=0))
    X = synth.stream_matrix(65536, 32, seed=1, missing_rate=0.02)
    c.score_matrix_oracle(X[:64])
    t = time.perf_counter()
    c.score_matrix_oracle(X)
    rate = len(X) / (time.perf_counter() - t)
    print(f"host 1000-tree GBDT: {rate:.0f} records/s")
    assert rate > 20_000


@pytest.mark.parametrize("shape", [dict(n_features=12, hidden=(40, 17)), dict(n_features=5, hidden=(8,), n_out=3,
                                                                             classification=True),
                                   dict(n_features=30, hidden=(64, 64, 32), activation="tanh")])
def test_native_neural_layers_are_bit_identical_to_the_connection_loop(shape):
    """nn_host.cpp::seq_affine: bias + products summed in connection order, one rounding each (no
    FMA) -- the numpy per-connection loop's exact bits."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix

    doc = mlp_pmml(seed=3, **shape)
    X = stream_matrix(700, shape["n_features"], seed=4, missing_rate=0.02)
    c1 = CompiledPmml.from_string(doc)
    assert all(e is not None for e in c1.evaluator._native_layers())
    s1, v1 = c1.score_matrix_oracle(X)
    c2 = CompiledPmml.from_string(doc)
    c2.evaluator._native = [None] * len(c2.evaluator.nn.layers)
    s2, v2 = c2.score_matrix_oracle(X)
    np.testing.assert_array_equal(v1, v2)
    assert np.array_equal(s1[v1], s2[v2])


def test_thread_count_does_not_change_results():
    """set_walk_threads / FJA_HOST_THREADS: blocks of rows on worker threads, every block writing
    only its own rows -- bit-identical results for any thread count."""
    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.native import fastpath

    c = CompiledPmml.from_string(_gbdt_doc(5, n_trees=64))
    prog = c.evaluator.native_forest()
    X = np.ascontiguousarray(synth.stream_matrix(50_000, 8, seed=2, missing_rate=0.05), dtype=np.float64)
    try:
        fastpath().set_walk_threads(1)
        one = (prog.leaves(X), prog.values(X), prog.sums(X))
        fastpath().set_walk_threads(6)
        six = (prog.leaves(X), prog.values(X), prog.sums(X))
    finally:
        fastpath().set_walk_threads(1)
    for a, b in zip(one, six):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction", "lastPrediction"])
@pytest.mark.parametrize("weighted", [False, True])
def test_native_majority_vote_equals_segment_loop(missing, weighted):
    """The native vote (one leaf walk + tree-order bincount) gives the per-segment ``_classify``
    loop's labels, validity and vote shares bit for bit."""
    from flink_jpmml_amd.bench import synth

    doc = synth.random_forest_pmml(n_trees=40, depth=7, n_features=10, n_classes=4, seed=3,
                                   missing_strategy=missing if missing != "lastPrediction" else "defaultChild")
    if missing == "lastPrediction":
        doc = doc.replace('missingValueStrategy="defaultChild"', 'missingValueStrategy="lastPrediction"')
    if weighted:
        doc = doc.replace('multipleModelMethod="majorityVote"', 'multipleModelMethod="weightedMajorityVote"')
        k = [0]

        def _w(m):
            k[0] += 1
            return f'<Segment id="{m.group(1)}" weight="{0.25 + (k[0] % 7) * 0.375}"'
        import re
        doc = re.sub(r'<Segment id="([^"]+)"', _w, doc)
    c = CompiledPmml.from_string(doc)
    ev = c.evaluator
    assert ev.native_vote() is not None
    X = synth.stream_matrix(3000, 10, seed=4, missing_rate=0.15)
    res_native = ev.evaluate(c.columns(c.prepare(X)[0]))
    prog, glab, offs, w, _ = ev.native_vote()
    L = prog.leaves(prog.matrix(c.columns(c.prepare(X)[0])))
    res_np = ev._vote_native(L, glab, offs, w)  # the numpy form of the same vote
    ev._native_vote = None  # the per-segment loop
    res_loop = ev.evaluate(c.columns(c.prepare(X)[0]))
    np.testing.assert_array_equal(res_native.valid, res_loop.valid)
    np.testing.assert_array_equal(res_native.value, res_loop.value)
    np.testing.assert_array_equal(res_native.probs, res_loop.probs)
    for r in (res_np,):
        np.testing.assert_array_equal(r.valid, res_loop.valid)
        np.testing.assert_array_equal(r.value, res_loop.value)
        np.testing.assert_array_equal(r.probs, res_loop.probs)
    assert res_native.valid.any() and (not res_native.valid.all() or missing == "defaultChild")
