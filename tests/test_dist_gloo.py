"""Multi-process data-parallel paths on the gloo backend (CPU, world size 2 and 4).

The RCCL path is the same code with backend ``nccl``; it runs on GPU boxes (the 8-GPU scaling run
is the driver's). These tests cover the collectives' semantics: control-plane replication,
tensor/plan payload broadcast, varlen all-gather, sharding and the distributed serving protocol.
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, res = q.get(timeout=120)
        results[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, res in results.items():
        if isinstance(res, BaseException):
            raise res
    return results


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from flink_jpmml_amd.parallel import init_from_env, shutdown

        ctx = init_from_env(backend="gloo")
        res = fn(ctx, *args)
        shutdown(ctx)
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, e))


# ---------------------------------------------------------------------------------- workers
def w_control(ctx):
    from flink_jpmml_amd.domain import AddMessage, DelMessage
    from flink_jpmml_amd.parallel import broadcast_control

    msgs = [AddMessage("f5c4e8b3-4a1e-4b3c-9b5e-123456789abc", 1, "/m.xml", 5),
            DelMessage("f5c4e8b3-4a1e-4b3c-9b5e-123456789abc", 1, 6)] if ctx.rank == 0 else None
    got = broadcast_control(msgs, ctx)
    empty = broadcast_control([] if ctx.rank == 0 else None, ctx)
    return [repr(m) for m in got], len(empty)


def w_tensors(ctx):
    import torch

    from flink_jpmml_amd.parallel import broadcast_tensors

    spec = {"a": ((3, 4), "float32"), "b": ((5,), "int32"), "c": ((2, 2), "uint8")}
    src = None
    if ctx.rank == 0:
        src = {"a": torch.arange(12, dtype=torch.float32).view(3, 4), "b": torch.arange(5, dtype=torch.int32) * 7,
               "c": torch.tensor([[1, 2], [3, 255]], dtype=torch.uint8)}
    out = broadcast_tensors(src, spec, ctx)
    return {k: v.tolist() for k, v in out.items()}


def w_gather(ctx):
    import torch

    from flink_jpmml_amd.parallel import all_gather_scores, all_gather_varlen, shard_range

    lo, hi = shard_range(10, ctx.rank, ctx.world_size)
    s, v, _ = all_gather_scores(torch.full((3,), float(ctx.rank)), torch.ones(3, dtype=torch.uint8), ctx)
    var = all_gather_varlen(torch.arange(lo, hi, dtype=torch.float32), ctx)
    return s.tolist(), var.tolist(), (lo, hi)


def w_serving(ctx, kmeans_path, notarget_path):
    from flink_jpmml_amd.domain import AddMessage, DelMessage
    from flink_jpmml_amd.parallel import shard_range
    from flink_jpmml_amd.parallel.serving import DistributedServing

    n1 = "a1b2c3d4-0000-4000-8000-000000000001"
    n2 = "a1b2c3d4-0000-4000-8000-000000000002"
    srv = DistributedServing(ctx)
    srv.apply_control([AddMessage(n1, 1, kmeans_path), AddMessage(n2, 1, notarget_path),
                       AddMessage(n1, 1, notarget_path)] if ctx.rank == 0 else None)
    X = np.tile(np.array([[1.0, 1.0, 1.0, 1.0], [1.0, 2.0, 3.0, 4.0]]), (5, 1))
    lo, hi = shard_range(len(X), ctx.rank, ctx.world_size)
    s1, v1 = srv.gather(*srv.score(f"{n1}_1", X[lo:hi]))
    s2, v2 = srv.gather(*srv.score(f"{n2}_1", X[lo:hi]))
    srv.apply_control([DelMessage(n1, 1)] if ctx.rank == 0 else None)
    s3, v3 = srv.gather(*srv.score(f"{n1}_1", X[lo:hi]))
    return s1.tolist(), v1.tolist(), v2.tolist(), v3.tolist(), sorted(str(k) for k in srv.metadata)


# ---------------------------------------------------------------------------------- tests
@pytest.mark.parametrize("world", [2, 4])
def test_control_plane_broadcast(world):
    res = _run(world, w_control)
    assert all(r == res[0] for r in res.values())
    assert "AddMessage" in res[0][0][0] and "DelMessage" in res[0][0][1] and res[0][1] == 0


def test_tensor_broadcast_single_buffer():
    res = _run(2, w_tensors)
    assert res[1] == res[0]
    assert res[1]["b"] == [0, 7, 14, 21, 28] and res[1]["c"] == [[1, 2], [3, 255]]


@pytest.mark.parametrize("world", [2, 3])
def test_gather_and_sharding(world):
    res = _run(world, w_gather)
    for r, (s, var, (lo, hi)) in res.items():
        assert s == [float(i) for i in range(world) for _ in range(3)]
        assert var == [float(i) for i in range(10)]
    shards = sorted(v[2] for v in res.values())
    assert shards[0][0] == 0 and shards[-1][1] == 10


def test_distributed_serving(fixtures_dir):
    res = _run(2, w_serving, fixtures_dir["kmeans"], fixtures_dir["kmeans_nooutput_notarget"])
    for s1, v1, v2, v3, meta in res.values():
        assert s1 == [3.0, 4.0] * 5 and all(v1)  # duplicate Add ignored on every rank
        assert not any(v2)  # model without a target -> EmptyScore everywhere
        assert not any(v3)  # deleted -> EmptyScore
        assert len(meta) == 1


# ------------------------------------------------------------------------------ tree sharding
def w_tree_shard(ctx, objective, missing):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.parallel import TreeShardedScorer
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=37, depth=5, n_features=10, seed=4, objective=objective,
                                           missing_strategy=missing))
    X = stream_matrix(2000, c.n_features, seed=5, missing_rate=0.03)
    ts = TreeShardedScorer(c, ctx)
    s, v = ts.score(X)
    return ts.n_trees_local, s.numpy(), v.numpy()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("objective,missing", [("regression", "defaultChild"), ("binary", "defaultChild"),
                                               ("regression", "nullPrediction")])
def test_tree_sharded_ensemble_matches_oracle(world, objective, missing):
    """TP over trees: each rank scores its slice, all_reduce(SUM/MIN) + epilogue == full model."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    res = _run(world, w_tree_shard, objective, missing)
    assert sum(r[0] for r in res.values()) == 37
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=37, depth=5, n_features=10, seed=4, objective=objective,
                                           missing_strategy=missing))
    X = stream_matrix(2000, c.n_features, seed=5, missing_rate=0.03)
    ref, vref = c.score_matrix_oracle(X)
    for r in range(world):
        _, s, v = res[r]
        assert (v == vref).all()
        if missing == "nullPrediction":
            assert not vref.all() and vref.any()
        if objective == "regression":
            np.testing.assert_allclose(s[vref], ref[vref], atol=2e-5)
        else:
            assert (s[vref] == ref[vref]).all()
        np.testing.assert_array_equal(s, res[0][1])


def test_tree_shard_rejects_multiclass():
    from flink_jpmml_amd.bench.synth import random_forest_pmml
    from flink_jpmml_amd.parallel import tree_shard_supported
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(random_forest_pmml(n_trees=4, depth=3, n_features=5, n_classes=3, seed=1))
    assert "single-score" in tree_shard_supported(c)


# ------------------------------------------------------------------ fault injection
def _kill_entry(rank, world, port, kmeans_path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FJA_FAULTS="kill_rank=1@2")
    from flink_jpmml_amd.domain import AddMessage
    from flink_jpmml_amd.parallel import init_from_env
    from flink_jpmml_amd.parallel.serving import DistributedServing
    from flink_jpmml_amd.utils.faults import RankFailure

    ctx = init_from_env(backend="gloo", timeout_s=20)
    srv = DistributedServing(ctx)
    name = "a1b2c3d4-0000-4000-8000-0000000000aa"
    srv.apply_control([AddMessage(name, 1, kmeans_path)] if rank == 0 else None)
    X = np.ones((3, 4))
    done = 0
    try:
        for _ in range(5):
            srv.gather(*srv.score(f"{name}_1", X))
            done += 1
        q.put((rank, ("finished", done)))
    except RankFailure as e:
        q.put((rank, ("rank-failure", done, str(e)[:200])))
    q.close()
    q.join_thread()  # flush the queue's feeder thread: os._exit would drop the pending message
    os._exit(0)


def test_killed_rank_surfaces_as_rank_failure(fixtures_dir):
    """kill_rank=1@2: rank 1 exits before its third micro-batch; rank 0's next all-gather raises
    RankFailure (not a hang) after exactly two completed batches."""
    from flink_jpmml_amd.utils.faults import EXIT_KILLED_RANK

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_kill_entry, args=(r, 2, port, fixtures_dir["kmeans"], q)) for r in range(2)]
    for p in procs:
        p.start()
    r, res = q.get(timeout=90)
    for p in procs:
        p.join(timeout=60)
    assert r == 0 and res[0] == "rank-failure" and res[1] == 2
    assert procs[1].exitcode == EXIT_KILLED_RANK


# ------------------------------------------------------------------ ADVICE r1 (tree-shard host path)
def _string_label_chain(n_trees, depth, F, seed):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    t = gbdt_pmml(n_trees=n_trees, depth=depth, n_features=F, seed=seed, objective="binary")
    t = t.replace('<DataField name="y" optype="categorical" dataType="integer">\n   <Value value="0"/>\n'
                  '   <Value value="1"/>', '<DataField name="y" optype="categorical" dataType="string">\n'
                  '   <Value value="no"/>\n   <Value value="yes"/>')
    t = t.replace('targetCategory="1"', 'targetCategory="yes"').replace('targetCategory="0"', 'targetCategory="no"')
    # a missingValueReplacement on f0 of the top-level schema: host ranks must prepare like the kernel
    return t.replace('<MiningField name="y" usageType="target"/>\n   <MiningField name="f0"/>',
                     '<MiningField name="y" usageType="target"/>\n   <MiningField name="f0" '
                     'missingValueReplacement="0.25"/>', 1)


def w_tree_shard_text(ctx, text):
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.parallel import TreeShardedScorer
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(text)
    X = stream_matrix(1500, c.n_features, seed=8, missing_rate=0.05)
    s, v = TreeShardedScorer(c, ctx).score(X)
    return s.numpy(), v.numpy()


def test_tree_shard_string_labels_and_missing_replacement():
    """String calibrator categories give EmptyScore (NaN label table, like the kernel) instead of
    a ValueError; host ranks apply MiningField missingValueReplacement before traversing."""
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.parallel import finish_epilogue
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    text = _string_label_chain(23, 4, 6, 3)
    c = CompiledPmml.from_string(text)
    assert c.mining_fields["f0"].missing_value_replacement is not None
    res = _run(2, w_tree_shard_text, text)
    X = stream_matrix(1500, c.n_features, seed=8, missing_rate=0.05)
    _, vref = c.score_matrix_oracle(X)
    for r in range(2):
        s, v = res[r]
        assert not v.any() and not vref.any()  # string labels are not numeric targets -> EmptyScore
    import torch

    s, ok = finish_epilogue(torch.zeros(3), torch.ones(3, dtype=torch.uint8), {"mode": 1, "a": 1.0, "b": 0.0,
                                                                               "link": 1}, ["no", "yes"])
    assert not ok.any()
    # numeric labels + the replacement: shard sums match the oracle exactly where f0 is missing
    num = text.replace('"yes"', '"1"').replace('"no"', '"0"').replace('dataType="string"', 'dataType="integer"')
    cn = CompiledPmml.from_string(num)
    res = _run(2, w_tree_shard_text, num)
    ref, vref = cn.score_matrix_oracle(X)
    assert vref.all() and np.isnan(X[:, 0]).any()
    for r in range(2):
        s, v = res[r]
        assert v.all() and (s == ref).all()


# ------------------------------------------------------------ model-sharded serving
def w_sharded(ctx, paths, X, ids_per_rank):
    from flink_jpmml_amd.domain import AddMessage, DelMessage
    from flink_jpmml_amd.parallel.serving import DistributedServing
    from flink_jpmml_amd.utils.metrics import METRICS

    srv = DistributedServing(ctx, placement="sharded")
    names = [f"a1b2c3d4-0000-4000-8000-{i:012d}" for i in range(len(paths))]
    srv.apply_control([AddMessage(n, 1, p) for n, p in zip(names, paths)] if ctx.rank == 0 else None)
    held = sorted(str(k) for k in srv.models)
    owners = {f"{n}_1": srv.owner(f"{n}_1") for n in names}
    ids = [f"{names[i]}_1" if i >= 0 else "ffffffff-0000-4000-8000-000000000000_1" for i in ids_per_rank[ctx.rank]]
    s, v = srv.score_routed(ids, X[ctx.rank])
    srv.apply_control([DelMessage(names[0], 1)] if ctx.rank == 0 else None)
    s2, v2 = srv.score_routed(ids, X[ctx.rank])
    routed = METRICS.summary().get("counters", {}).get("serving.routed_rows", 0)
    return held, owners, s.tolist(), v.tolist(), v2.tolist(), routed


@pytest.mark.parametrize("world", [2, 3])
def test_model_sharded_serving_routes_to_owner(world, tmp_path):
    """Every model is held by exactly one rank; mixed-model batches arriving on any rank are
    routed to the owners (all_to_all), scored and returned in arrival order == the oracle."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    txts = [gbdt_pmml(n_trees=5, depth=3, n_features=6, seed=s) for s in range(4)] + \
        [random_forest_pmml(n_trees=5, depth=3, n_features=6, n_classes=3, seed=9)]
    paths = []
    for i, t in enumerate(txts):
        p = tmp_path / f"m{i}.pmml"
        p.write_text(t)
        paths.append(str(p))
    rng = np.random.default_rng(0)
    X = [stream_matrix(40 + 7 * r, 6, seed=r) for r in range(world)]
    ids = [rng.integers(-1, len(paths), len(x)).tolist() for x in X]
    res = _run(world, w_sharded, paths, X, ids)
    held_all = sorted(m for r in res.values() for m in r[0])
    assert len(held_all) == len(paths) and len(set(held_all)) == len(paths)  # one owner per model
    owners = res[0][1]
    for r, (held, own, s, v, v2, routed) in res.items():
        assert own == owners and all(owners[m] == r for m in held)
        s, v, v2 = np.array(s), np.array(v), np.array(v2)
        for i, code in enumerate(ids[r]):
            if code < 0:
                assert not v[i]
                continue
            ref, vref = CompiledPmml.from_string(txts[code]).score_matrix_oracle(X[r][i:i + 1])
            assert v[i] == vref[0]
            assert s[i] == pytest.approx(ref[0], abs=1e-6)  # float32 score buffers
            assert v2[i] == (vref[0] and code != 0)  # model 0 deleted everywhere
        assert routed > 0


def w_evict(ctx, paths):
    from flink_jpmml_amd.domain import AddMessage
    from flink_jpmml_amd.parallel.serving import DistributedServing
    from flink_jpmml_amd.utils.metrics import METRICS

    METRICS.reset()
    srv = DistributedServing(ctx, cache_capacity=1)
    names = [f"a1b2c3d4-0000-4000-8000-{i:012d}" for i in range(2)]
    srv.apply_control([AddMessage(n, 1, p) for n, p in zip(names, paths)] if ctx.rank == 0 else None)
    X = np.tile(np.array([[1.0, 1.0, 1.0, 1.0], [1.0, 2.0, 3.0, 4.0]]), (3, 1))
    out = [srv.score(f"{names[i]}_1", X)[0].tolist() for i in (0, 1, 0)]
    c = METRICS.summary()["counters"]
    return out, c.get("serving.cache_misses", 0), c.get("serving.cache_evictions", 0)


def test_serving_cache_eviction_reloads(fixtures_dir):
    res = _run(2, w_evict, [fixtures_dir["kmeans"], fixtures_dir["kmeans"]])
    for out, misses, evictions in res.values():
        assert out[0] == out[2] == [3.0, 4.0] * 3
        assert misses >= 2 and evictions >= 2
