"""The LTOP pointer walk (the default for deep forests: levels 0-4 of every lock-step group's trees
staged in LDS, `tree.hip::pointer_walk<..., LTOP>`) across the shapes its LDS carve and staging
depend on: feature counts (LDS planes of 8 to 64 features), 1 to 12 class slots (GENERAL
accumulators before the staged nodes), a tree count that is not a multiple of the 8-tree group
(empty slots in the last group; the blob's zero padding), shallow and deep trees, both missing
strategies, and row counts that are not a multiple of the 256-row tile. Every plan must equal the
clamped lock-step walk bit for bit and the fp64 oracle in validity."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml

pytestmark = pytest.mark.gpu

CASES = [
    # kind, n_trees, depth, n_features, classes, p_split, missing, rows
    ("gbdt", 37, 13, 8, 1, 0.8, "defaultChild", 10_007),
    ("gbdt", 64, 15, 64, 1, 0.85, "nullPrediction", 20_000),
    ("gbdt", 9, 12, 33, 1, 0.5, "defaultChild", 777),
    ("rf", 30, 14, 16, 5, 0.8, "defaultChild", 9_000),
    ("rf", 21, 13, 24, 12, 0.75, "nullPrediction", 5_001),
    ("rf", 8, 16, 48, 2, 0.85, "defaultChild", 3_000),
]


def _scores(plan, X):
    import torch

    Xd = torch.from_numpy(X).cuda()
    s, v = plan.alloc_outputs(len(X))
    plan.launch(Xd, s, v)
    torch.cuda.synchronize()
    return s.cpu().numpy(), v.cpu().numpy().astype(bool)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-t{c[1]}-d{c[2]}-f{c[3]}-c{c[4]}")
def test_ltop_walk_equals_clamped_walk_and_oracle(gpu, case):
    from flink_jpmml_amd.runtime.plans import VAR_POINTER_LTOP

    kind, n_trees, depth, F, C, p_split, missing, rows = case
    if kind == "gbdt":
        doc = gbdt_pmml(n_trees=n_trees, depth=depth, n_features=F, seed=n_trees, p_split=p_split,
                        missing_strategy=missing)
    else:
        doc = random_forest_pmml(n_trees=n_trees, depth=depth, n_features=F, n_classes=C, seed=n_trees,
                                 p_split=p_split, missing_strategy=missing)
    c = CompiledPmml.from_string(doc)
    ltop = c.plan(gpu, layout="pointer")
    ref_plan = c.plan(gpu, layout="pointer", pointer_load="clamped")
    assert ltop.variant == VAR_POINTER_LTOP and ref_plan.variant == 0
    X = stream_matrix(rows, F, seed=rows, missing_rate=0.04)
    s, v = _scores(ltop, X)
    s0, v0 = _scores(ref_plan, X)
    assert (v == v0).all() and np.array_equal(s[v], s0[v0])
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if kind == "gbdt":
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=5e-5)
    else:
        np.testing.assert_array_equal(s[v], ref[v])


@pytest.mark.parametrize("opts", [dict(xcd_split="on"), dict(splits=3)], ids=["xcd", "splits3"])
@pytest.mark.parametrize("kind", ["gbdt", "rf"])
def test_ltop_walk_with_tree_splits(gpu, opts, kind):
    """Tree slices per workgroup (XCD-aware slices, grid.y splits + the split reduction): every
    slice stages its own groups' top levels."""
    from flink_jpmml_amd.runtime.plans import VAR_POINTER_LTOP

    if kind == "gbdt":
        doc = gbdt_pmml(n_trees=70, depth=13, n_features=20, seed=5, p_split=0.8)
    else:
        doc = random_forest_pmml(n_trees=45, depth=13, n_features=20, n_classes=3, seed=5, p_split=0.8)
    c = CompiledPmml.from_string(doc)
    plan = c.plan(gpu, layout="pointer", **opts)
    ref_plan = c.plan(gpu, layout="pointer", pointer_load="clamped", **opts)
    assert plan.variant == VAR_POINTER_LTOP
    X = stream_matrix(12_345, 20, seed=6, missing_rate=0.03)
    s, v = _scores(plan, X)
    s0, v0 = _scores(ref_plan, X)
    assert (v == v0).all() and np.array_equal(s[v], s0[v0])
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
