"""LDS-resident deep-forest walk (``ops/csrc/tree_lds.hip``, ``TreePlan(node_format="lds")``):
the chunk tables cover every tree exactly once in order, slice by slice, every chunk fits the
LDS buffer, and a numpy emulation of the kernel — chunks copied from their even slot start into a
local buffer, trees walked with chunk-local positions, thread-group / slice summation order —
reproduces the float64 oracle (CPU, dry-run plans). GPU twin: ``test_gpu_lds_forest.py``."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.hybrid import pack_lds_chunks
from flink_jpmml_amd.runtime.plans import VAR_POINTER_LDS, TreePlan, lowering_dry_run


def _plan(txt, **kw):
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        return c, TreePlan(c, torch.device("cpu"), layout="pointer", node_format="lds", **kw)


def check_tables(plan):
    chunks = plan.lds_chunks.numpy().reshape(-1, 4)
    slices = plan.lds_slices.numpy()
    roots = plan.roots.numpy().astype(np.int64)
    start = np.where(roots >= 0, roots, ~roots)
    n_slots = plan.blob.numpy().size // 2
    end = np.append(start[1:], n_slots)
    assert slices[0] == 0 and slices[-1] == len(chunks) and (np.diff(slices) >= 1).all()
    assert chunks[0, 2] == 0 and chunks[-1, 3] == plan.n_trees and (chunks[1:, 2] == chunks[:-1, 3]).all()
    for x, u4, tb, te in chunks.tolist():
        assert x % 2 == 0 and u4 <= plan.lds_chunk_u4 and te > tb
        assert x <= start[tb] and end[te - 1] <= x + 2 * u4  # every tree of the chunk is in the copy


def emulate_lds(plan, X):
    """tree_lds_kernel, P = 1 sums: per slice, per chunk, the group's trees in order; groups and
    slices added in order (fp32 like the kernel)."""
    Xf = X.astype(np.float32)
    n = len(X)
    blob = plan.blob.numpy().view(np.uint32).reshape(-1, 2)
    roots = plan.roots.numpy().astype(np.int64)
    chunks = plan.lds_chunks.numpy().reshape(-1, 4)
    slices = plan.lds_slices.numpy()
    G = 1024 // plan.lds_rows
    total = np.zeros(n, np.float32)
    for s in range(len(slices) - 1):
        part = np.zeros((G, n), np.float32)
        for c in range(slices[s], slices[s + 1]):
            x0, u4, tb, te = chunks[c].tolist()
            local = blob[x0: x0 + 2 * u4]
            for t in range(tb, te):
                g = (t - tb) % G
                r = roots[t]
                pos = np.full(n, (r if r >= 0 else ~r) - x0, np.int64)
                act = np.full(n, r >= 0)
                pz = np.zeros(n, bool)
                while act.any():
                    nd = local[np.where(act, pos, 0)]
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
                val = local[pos, 0].view(np.float32)
                part[g] += np.where(pz, np.float32(np.nan), val)
        acc = part[0].copy()
        for g in range(1, G):
            acc += part[g]
        total += acc
    return total


def test_pack_lds_chunks_slices_and_limits():
    roots = np.array([0, 10, 25, 26, 40, 100], dtype=np.int32)  # tree 3 is a one-slot tree
    chunks, slices = pack_lds_chunks(130, roots, chunk_u4=32, n_slices=2)
    assert slices.tolist()[0] == 0 and slices[-1] == len(chunks) and len(slices) == 3
    assert chunks[:, 2].tolist()[0] == 0 and chunks[-1, 3] == 6
    assert (chunks[:, 1] <= 32).all() and (chunks[:, 0] % 2 == 0).all()
    with pytest.raises(ValueError):
        pack_lds_chunks(130, roots, chunk_u4=20, n_slices=2)  # tree 4 (60 slots) cannot fit


@pytest.mark.parametrize("missing", ["defaultChild", "nullPrediction"])
def test_lds_walk_matches_oracle(missing):
    txt = gbdt_pmml(n_trees=40, depth=12, n_features=24, seed=3, p_split=0.8)
    if missing == "nullPrediction":
        txt = txt.replace('missingValueStrategy="defaultChild"', 'missingValueStrategy="nullPrediction"')
    c, plan = _plan(txt)
    assert plan.variant == VAR_POINTER_LDS and plan.layout == "pointer" and plan.lds_n_slices == 8
    check_tables(plan)
    X = stream_matrix(3000, 24, seed=5, missing_rate=0.03)
    ref, vref = c.score_matrix_oracle(X)
    got = plan.epi_args.get("a", 1.0) * emulate_lds(plan, X).astype(np.float64) + plan.epi_args.get("b", 0.0)
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], rtol=0, atol=2e-4)


def test_lds_tables_for_deep_forests_and_votes():
    """300-tree-class sizes: depth-14 trees of ~5000 slots fit 512-row tiles; a random forest
    (class votes, GENERAL) lowers too; the plan is not offered to the grouped / batched launchers."""
    c, plan = _plan(gbdt_pmml(n_trees=24, depth=14, n_features=32, seed=0, p_split=0.85))
    check_tables(plan)
    assert plan.lds_rows == 512 and plan.batch_launch_args(0, 10, 32, 32, 0, 0) is None
    c, rf = _plan(random_forest_pmml(n_trees=16, depth=12, n_features=32, n_classes=3, seed=1))
    assert rf.general == 1 and rf.variant == VAR_POINTER_LDS
    check_tables(rf)
