"""Tree-sharded ensembles on the HIP kernels: raw per-shard sums from ``TreePlan(tree_shard=...)``
combined as the RCCL ``all_reduce`` would (sum of partials, min of valid bytes) and finished by the
torch epilogue must equal the unsharded kernel and the float64 oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("objective,missing,world", [("regression", "defaultChild", 3),
                                                     ("binary", "defaultChild", 2),
                                                     ("regression", "nullPrediction", 4)])
def test_tree_shards_combine_to_full_model(gpu, objective, missing, world):
    import torch

    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.parallel import DistContext, TreeShardedScorer, finish_epilogue
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=301, depth=6, n_features=24, seed=7, objective=objective,
                                           missing_strategy=missing))
    X = stream_matrix(20000, c.n_features, seed=8, missing_rate=0.02)
    ref, vref = c.score_matrix_oracle(X)
    Xt = torch.from_numpy(X.astype(np.float32)).to(gpu)
    raw = torch.zeros(len(X), device=gpu)
    valid = torch.ones(len(X), dtype=torch.uint8, device=gpu)
    n = 0
    for r in range(world):
        p = TreePlan(c, gpu, tree_shard=(r, world))
        n += p.n_trees
        s, v = p.alloc_outputs(len(X))
        p.launch(Xt, s, v)
        raw += torch.where(v.bool(), s, torch.zeros_like(s))
        valid = torch.minimum(valid, v)
    assert n == 301
    s, v = finish_epilogue(raw, valid, p.full_epi, p.labels)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    assert (v == vref).all()
    full_s, full_v = TreePlan(c, gpu).score(X)
    assert (full_v.cpu().numpy() == v).all()
    if objective == "regression":
        np.testing.assert_allclose(s[v], ref[v], atol=3e-5)
    else:
        assert (s[v] == ref[v]).all()
    # world-size-1 scorer (no collective) is the unsharded model
    one = TreeShardedScorer(c, DistContext(device=gpu))
    s1, v1 = one.score(X)
    assert (v1.cpu().numpy() == vref).all()
