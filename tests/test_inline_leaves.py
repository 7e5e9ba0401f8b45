"""Inline leaf payloads on the lock-step pointer walk (``VAR_POINTER_INLINE``,
``runtime/hybrid.py::pack_trees(inline_leaves=True)``, ``tree.hip::pointer_walk<..., INL>``): a
leaf child's payload sits in its parent's child field (meta bit 29 left / 28 right) -- the fp32
leaf value of a sum ensemble, the class index of a unit vote -- so the walk needs no leaf gather.
CPU: a numpy twin of the walk over the packed nodes equals the leaf-table walk and the oracle;
GPU: the kernel is bit-identical to the table walk and matches the oracle."""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.hybrid import INLINE_LEFT_BIT, INLINE_RIGHT_BIT, pack_trees
from flink_jpmml_amd.runtime.plans import TB, ensemble_spec, to_general


def _walk(nodes, leaves, roots, X, P, inline):
    """numpy twin of pointer_walk (features from X directly; meta offsets are byte offsets into
    the [F][TB] LDS planes)."""
    n = len(X)
    Xf = X.astype(np.float32)
    acc = np.zeros((n, P), dtype=np.float64)
    poisoned = np.zeros(n, dtype=bool)
    for r in range(n):
        for root in roots:
            code, pay, done_inline = int(root), 0, False
            while code >= 0:
                T, meta, lc, rc = (int(v) for v in nodes[code])
                f = (meta & 0xFFFF) // (TB * 4)
                x = Xf[r, f]
                isn = np.isnan(x)
                if isn and (meta >> 30) & 1:
                    poisoned[r] = True
                    code = -1
                    break
                right = bool(x >= np.uint32(T).view(np.float32)) or (isn and (meta >> 31) & 1)
                child = rc if right else lc
                if inline and (meta >> (INLINE_RIGHT_BIT if right else INLINE_LEFT_BIT)) & 1:
                    pay, done_inline, code = child, True, -1
                    break
                code = int(np.int32(np.uint32(child)))
            if poisoned[r]:
                continue
            if done_inline:
                if P == 1:
                    acc[r, 0] += float(np.uint32(pay).view(np.float32))
                else:
                    acc[r, pay] += 1.0
            else:
                acc[r] += leaves[~code]
    acc[poisoned] = np.nan
    return acc


@pytest.mark.parametrize("kind,missing", [("gbdt", "defaultChild"), ("gbdt", "nullPrediction"), ("rf", "none")])
def test_inline_twin_equals_table_and_oracle(kind, missing):
    if kind == "gbdt":
        txt = gbdt_pmml(n_trees=9, depth=7, n_features=6, seed=3, p_split=0.8, missing_strategy=missing)
    else:
        txt = random_forest_pmml(n_trees=9, depth=7, n_features=6, n_classes=3, seed=4, p_split=0.8)
    c = CompiledPmml.from_string(txt)
    spec = to_general(ensemble_spec(c))
    P = spec.P
    X = stream_matrix(400, 6, seed=5, missing_rate=0.05)
    _, n0, l0, r0, _ = pack_trees(spec.trees, spec.weights, P, 0, True)
    _, n1, l1, r1, _ = pack_trees(spec.trees, spec.weights, P, 0, True, inline_leaves=True)
    assert (n1[:, 1] & ((1 << INLINE_LEFT_BIT) | (1 << INLINE_RIGHT_BIT))).any()
    a0 = _walk(n0, l0, r0, X, P, False)
    a1 = _walk(n1, l1, r1, X, P, True)
    np.testing.assert_array_equal(np.isnan(a0), np.isnan(a1))
    np.testing.assert_allclose(np.nan_to_num(a1), np.nan_to_num(a0), rtol=0, atol=1e-6)
    ref, vref = c.score_matrix_oracle(X)
    ok = ~np.isnan(a1).any(axis=1)
    assert (ok == vref).all()
    if kind == "gbdt":
        e = spec.epi
        np.testing.assert_allclose(e["a"] * a1[ok, 0] + e["b"], ref[ok], rtol=0, atol=2e-5)
    else:
        lab = np.array([float(x) for x in spec.labels])[np.argmax(a1[ok], axis=1)]
        assert (lab == ref[ok]).mean() > 0.995  # ties broken the same way except within fp32


@pytest.mark.gpu
@pytest.mark.parametrize("load", ["auto", "ltop"])
@pytest.mark.parametrize("kind", ["gbdt", "rf"])
def test_inline_leaves_on_gpu(gpu, kind, load):
    import torch

    if kind == "gbdt":
        txt = gbdt_pmml(n_trees=60, depth=14, n_features=24, seed=7, p_split=0.8, missing_strategy="defaultChild")
        F = 24
    else:
        txt = random_forest_pmml(n_trees=40, depth=14, n_features=16, n_classes=3, seed=5, p_split=0.8)
        F = 16
    c = CompiledPmml.from_string(txt)
    inl = c.plan(gpu, layout="pointer", pointer_leaf="inline", pointer_load=load)
    tab = c.plan(gpu, layout="pointer", pointer_leaf="table")
    # inline leaves: the clamped walk (auto), or with the LDS-staged top levels; table leaves: LTOP
    assert inl.variant == (4096 if load == "auto" else 4096 | 8192) and tab.variant == 8192
    X = stream_matrix(100_000, F, seed=3, missing_rate=0.03)
    Xd = torch.from_numpy(X).cuda()
    outs = []
    for plan in (inl, tab):
        s, v = plan.alloc_outputs(len(X))
        plan.launch(Xd, s, v)
        torch.cuda.synchronize()
        outs.append((s.cpu().numpy(), v.cpu().numpy().astype(bool)))
    (s1, v1), (s0, v0) = outs
    assert (v1 == v0).all() and np.array_equal(s1[v1], s0[v0])  # same tree-order sums
    ref, vref = c.score_matrix_oracle(X)
    assert (v1 == vref).all()
    if kind == "gbdt":
        np.testing.assert_allclose(s1[v1], ref[v1], rtol=0, atol=5e-5)
    else:
        np.testing.assert_array_equal(s1[v1], ref[v1])
