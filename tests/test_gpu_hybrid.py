"""Deep forests on the MI355X: HYBRID layout (PERFECT head in LDS + POINTER tail) and the
vectorised POINTER layout against the float64 oracle, incl. an unbounded-depth (depth-20)
sklearn-style forest."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml

pytestmark = pytest.mark.gpu

# The deep documents take seconds to generate and parse, and their oracle scores are the same
# for every kernel variant: parse each once per session, score each input set once.
_MODELS: dict = {}
_ORACLE: dict = {}


def _model(kind: str, as_bytes: bool = False, **kw) -> CompiledPmml:
    key = (kind, as_bytes, tuple(sorted(kw.items())))
    c = _MODELS.get(key)
    if c is None:
        txt = (gbdt_pmml if kind == "gbdt" else random_forest_pmml)(**kw)
        c = _MODELS[key] = CompiledPmml.from_string(txt.encode() if as_bytes else txt)
    return c


def _oracle(c: CompiledPmml, X: np.ndarray):
    k = (id(c), id(X))  # both objects live in the caches for the whole session
    r = _ORACLE.get(k)
    if r is None:
        r = _ORACLE[k] = c.score_matrix_oracle(X)
    return r


def _inputs(n: int, f: int, seed: int, missing_rate: float) -> np.ndarray:
    k = ("X", n, f, seed, missing_rate)
    X = _ORACLE.get(k)
    if X is None:
        X = _ORACLE[k] = stream_matrix(n, f, seed=seed, missing_rate=missing_rate)
    return X


def _score(c, plan, X):
    import torch

    Xd = torch.from_numpy(X.astype(np.float32)).cuda()
    s, v = plan.alloc_outputs(len(X))
    plan.launch(Xd, s, v)
    torch.cuda.synchronize()
    return s.cpu().numpy(), v.cpu().numpy().astype(bool)


@pytest.mark.parametrize("layout,head", [("hybrid", 8), ("hybrid", 6), ("hybrid", 10), ("pointer", 0)])
@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
def test_deep_gbdt_on_gpu(gpu, layout, head, missing):
    c = _model("gbdt", n_trees=40, depth=14, n_features=24, seed=7, p_split=0.8, missing_strategy=missing)
    plan = c.plan(gpu, layout=layout, head_depth=head)
    assert plan.layout == layout
    X = _inputs(100_000, 24, 3, 0.03)
    s, v = _score(c, plan, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=5e-5)


@pytest.mark.parametrize("depth", [14, 20])
def test_deep_random_forest_votes_on_gpu(gpu, depth):
    """sklearn RandomForest with max_depth=None: majority vote over deep unbalanced trees; the
    depth-20 document goes through the streaming parser (flat arrays) as well."""
    c = _model("rf", True, n_trees=6 if depth == 20 else 30, depth=depth, n_features=16, n_classes=3, seed=5,
               p_split=0.8)
    plan = c.plan(gpu)
    assert plan.layout == "pointer" and plan.depth == depth
    X = _inputs(50_000, 16, 8, 0.02)
    s, v = _score(c, plan, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_array_equal(s[v], ref[v])


def test_wide_feature_deep_forest_global_features(gpu):
    """n_features > 64: the hybrid walk reads features from global memory (indices in the metas)."""
    c = _model("gbdt", n_trees=20, depth=12, n_features=90, seed=4)
    X = _inputs(30_000, 90, 2, 0.02)
    ref, vref = _oracle(c, X)
    for layout in ("hybrid", "pointer"):
        plan = c.plan(gpu, layout=layout)
        s, v = _score(c, plan, X)
        assert (v == vref).all()
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=5e-5)


@pytest.mark.parametrize("opts", [dict(layout="pointer"), dict(layout="pointer", node_format="compact"),
                                  dict(layout="pointer", pointer_schedule="refill"),
                                  dict(layout="hybrid", head_depth=4)])
@pytest.mark.parametrize("n_rows", [100_000, 777])
def test_xcd_split_forest_on_gpu(gpu, opts, n_rows):
    """XCD-aware tree slices (csrc ``tree_block``: workgroup L scores slice L % 8 of row block
    L / 8) against the fp64 oracle and against the unsplit launch, incl. a ragged last row block."""
    c = _model("gbdt", n_trees=40, depth=14, n_features=24, seed=11, p_split=0.8)
    X = _inputs(n_rows, 24, 4, 0.03)
    ref, vref = _oracle(c, X)
    on = c.plan(gpu, xcd_split="on", **opts)
    off = c.plan(gpu, xcd_split="off", **opts)
    assert on.xcd_split == 8 and off.xcd_split == 0 and on._auto_splits(n_rows) == 8
    s1, v1 = _score(c, on, X)
    s0, v0 = _score(c, off, X)
    assert (v1 == vref).all() and (v0 == vref).all()
    np.testing.assert_allclose(s1[v1], ref[v1], rtol=0, atol=5e-5)
    np.testing.assert_allclose(s1[v1], s0[v0], rtol=0, atol=5e-5)


def test_xcd_split_vote_forest_on_gpu(gpu):
    """Random-forest votes (P = 3 class slots accumulated in LDS) over XCD slices."""
    c = _model("rf", n_trees=48, depth=14, n_features=16, n_classes=3, seed=9, p_split=0.8)
    X = _inputs(60_000, 16, 1, 0.02)
    ref, vref = _oracle(c, X)
    plan = c.plan(gpu, layout="pointer", xcd_split="on")
    s, v = _score(c, plan, X)
    assert (v == vref).all()
    np.testing.assert_array_equal(s[v], ref[v])


@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
@pytest.mark.parametrize("xcd", ["off", "on"])
def test_super_layout_on_gpu(gpu, missing, xcd):
    """Two levels per 16-byte slot (tree_super_kernel): against the fp64 oracle, and bit-identical
    to the one-level pointer walk (both accumulate leaves in tree order)."""
    c = _model("gbdt", n_trees=40, depth=14, n_features=24, seed=7, p_split=0.8, missing_strategy=missing)
    sup = c.plan(gpu, layout="pointer", node_format="super", xcd_split=xcd)
    ptr = c.plan(gpu, layout="pointer", xcd_split=xcd)
    assert sup.variant == 128
    X = _inputs(100_000, 24, 3, 0.03)
    s, v = _score(c, sup, X)
    s0, v0 = _score(c, ptr, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=5e-5)
    assert (v == v0).all() and np.array_equal(s[v], s0[v0])


def test_super_layout_votes_on_gpu(gpu):
    c = _model("rf", True, n_trees=30, depth=16, n_features=16, n_classes=3, seed=5, p_split=0.8)
    plan = c.plan(gpu, layout="pointer", node_format="super")
    X = _inputs(50_000, 16, 8, 0.02)
    s, v = _score(c, plan, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_array_equal(s[v], ref[v])


@pytest.mark.parametrize("opts", [dict(layout="pointer", pointer_load="uskip"),
                                  dict(layout="pointer", pointer_load="peel"),
                                  dict(layout="pointer", pointer_load="ltop"),
                                  dict(layout="pointer", pointer_load="uskip", pointer_ilp=4),
                                  dict(layout="hybrid", hybrid_tail="wide", head_depth=2),
                                  dict(layout="hybrid", hybrid_tail="wide", head_depth=4, pointer_load="uskip"),
                                  dict(layout="hybrid", hybrid_tail="wide", head_depth=4),
                                  dict(layout="hybrid", hybrid_tail="wide", head_depth=3)])
@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
def test_uniform_skip_walks_on_gpu(gpu, opts, missing):
    """Wave-uniform skip of finished walk slots (pointer walk and the LDS-head + 16-byte pointer
    tail hybrid): against the fp64 oracle, and bit-identical to the clamped pointer walk (same
    tree-order leaf sums)."""
    c = _model("gbdt", n_trees=45, depth=14, n_features=24, seed=7, p_split=0.8, missing_strategy=missing)
    plan = c.plan(gpu, **opts)
    ptr = c.plan(gpu, layout="pointer", pointer_load="clamped")
    assert plan.layout == opts["layout"]
    X = _inputs(100_000, 24, 3, 0.03)
    s, v = _score(c, plan, X)
    s0, v0 = _score(c, ptr, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=5e-5)
    assert (v == v0).all() and np.array_equal(s[v], s0[v0])


@pytest.mark.parametrize("opts", [dict(layout="pointer", pointer_load="uskip"),
                                  dict(layout="pointer", pointer_load="peel"),
                                  dict(layout="pointer", pointer_load="ltop"),
                                  dict(layout="hybrid", hybrid_tail="wide", head_depth=3)])
def test_uniform_skip_votes_on_gpu(gpu, opts):
    """Random-forest votes (P = 3 class slots in LDS) on the uniform-skip walks."""
    c = _model("rf", True, n_trees=30, depth=16, n_features=16, n_classes=3, seed=5, p_split=0.8)
    plan = c.plan(gpu, **opts)
    X = _inputs(50_000, 16, 8, 0.02)
    s, v = _score(c, plan, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    np.testing.assert_array_equal(s[v], ref[v])


@pytest.mark.parametrize("load", ["peel", "ltop", "auto"])
@pytest.mark.parametrize("p_split", [0.35, 0.6])
def test_peeled_walks_with_shallow_leaves_on_gpu(gpu, load, p_split):
    """The peeled top levels when leaves sit at levels 1-2 (a leaf child of the root in most
    trees): bit-identical to the clamped walk, exact validity vs the oracle."""
    c = _model("gbdt", n_trees=64, depth=12, n_features=16, seed=11, p_split=p_split,
               missing_strategy="nullPrediction")
    plan = c.plan(gpu, layout="pointer", pointer_load=load)
    ptr = c.plan(gpu, layout="pointer", pointer_load="clamped")
    X = _inputs(60_000, 16, 4, 0.03)
    s, v = _score(c, plan, X)
    s0, v0 = _score(c, ptr, X)
    ref, vref = _oracle(c, X)
    assert (v == vref).all()
    assert (v == v0).all() and np.array_equal(s[v], s0[v0])
