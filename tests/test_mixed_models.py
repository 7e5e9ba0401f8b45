"""Mixed-model columnar batches in dynamic serving.

The reference serves many models from one operator, picking the model per event
(`S/package.scala:107-119`, `S/api/functions/EvaluationCoFunction.scala:106-117`). A RecordBatch
whose rows name different models (``model_ids``, plain or dictionary-encoded) is grouped in linear
time (native dictionary encoding + counting sort) and, on a GPU, scored in one grouped pass
(``runtime/grouped.py``, GPU tests below). Every row must equal the per-record prediction of its
own model."""

import math
import time

import numpy as np
import pytest

from flink_jpmml_amd import AddMessage, DelMessage, ModelReader
from flink_jpmml_amd.api.batch import RecordBatch
from flink_jpmml_amd.api.pmml_model import PmmlModel
from flink_jpmml_amd.bench import synth
from flink_jpmml_amd.config import ScoringConfig
from flink_jpmml_amd.stream import StreamExecutionEnvironment

UUIDS = [f"a1b2c3d4-0000-4000-8000-{k:012d}" for k in range(8)]


def _models(tmp_path, k=4, n_features=8):
    paths = []
    for i in range(k):
        p = tmp_path / f"m{i}.pmml"
        if i % 2:
            p.write_text(synth.gbdt_pmml(n_trees=12, depth=4, n_features=n_features, seed=i))
        else:
            p.write_text(synth.random_forest_pmml(n_trees=6, depth=4, n_features=n_features, n_classes=3, seed=i))
        paths.append(str(p))
    return paths


def test_group_rows_is_linear_and_exact():
    rng = np.random.default_rng(0)
    ids = [f"{u}_1" for u in UUIDS]
    n = 1 << 20
    col = np.array(ids, dtype=object)[rng.integers(0, len(ids), n)]
    dt = math.inf
    for _ in range(3):  # best of 3 (fresh batches: id codes are cached): a loaded host must not fail the rate check
        b = RecordBatch(np.zeros((n, 2), np.float32), model_ids=col)
        t = time.perf_counter()
        keys, perm, starts = b.group_rows()
        dt = min(dt, time.perf_counter() - t)
    assert sorted(keys) == sorted(ids) and starts[-1] == n
    for k, key in enumerate(keys):
        rows = perm[starts[k]:starts[k + 1]]
        assert (np.diff(rows) > 0).all() and (col[rows] == key).all()
    assert n / dt > 30e6, f"{n / dt / 1e6:.1f} M rows/s"  # ~100-300 M rows/s when the box is idle


def test_encoded_ids_round_trip():
    codes = np.array([2, 0, 1, 2, 2], dtype=np.uint8)
    b = RecordBatch(np.arange(10, dtype=np.float32).reshape(5, 2), model_ids=(codes, ["a", "b", "c"]))
    assert b.model_ids.tolist() == ["c", "a", "b", "c", "c"]
    subs = {s.model_id: s for s in b.split_by_model()}
    assert subs["c"].row_index.tolist() == [0, 3, 4] and subs["c"].X[:, 0].tolist() == [0.0, 6.0, 8.0]


@pytest.mark.parametrize("encoded", [False, True])
def test_dynamic_quick_evaluate_mixed_batch_matches_per_model(tmp_path, encoded):
    paths = _models(tmp_path, k=4)
    rng = np.random.default_rng(3)
    n = 3000
    X = synth.stream_matrix(n, 8, seed=4, missing_rate=0.05)
    # 4 served models + one id never added (EmptyScore rows)
    ids = [f"{UUIDS[i]}_1" for i in range(5)]
    code = rng.integers(0, 5, n)
    mids = (code.astype(np.uint8), ids) if encoded else np.array(ids, dtype=object)[code]
    seq = [("R", AddMessage(UUIDS[i], 1, paths[i], 0)) for i in range(4)] + \
          [("L", RecordBatch(X, model_ids=mids))] + [("R", DelMessage(UUIDS[0], 1, 0))] + \
          [("L", RecordBatch(X[:100], model_id=ids[0]))]
    env = StreamExecutionEnvironment()
    ev, ctrl = env.from_either(seq)
    out = ev.with_support_stream(ctrl).quick_evaluate().collect()
    assert len(out) == 2
    pb, batch = out[0]
    assert len(pb) == n and batch is not None
    for i in range(5):
        rows = np.flatnonzero(code == i)
        if i == 4:
            assert not pb.valid[rows].any()
            continue
        ref = PmmlModel.from_path(paths[i]).predict(X[rows])
        assert (pb.valid[rows] == ref.valid).all()
        np.testing.assert_array_equal(pb.scores[rows][ref.valid], ref.scores[ref.valid])
    assert not out[1][0].valid.any()  # deleted model: EmptyScore


def test_mixed_batch_with_wrong_width_model_is_empty_score(tmp_path):
    """on the split path a served model whose active-field count differs from the
    batch width scores EmptyScore rows (as the grouped path's NullScorer does), never raises."""
    paths = _models(tmp_path, k=2)
    narrow = tmp_path / "narrow.pmml"
    narrow.write_text(synth.gbdt_pmml(n_trees=4, depth=3, n_features=4, seed=9))
    n = 600
    X = synth.stream_matrix(n, 8, seed=1, missing_rate=0.0)
    code = np.arange(n) % 3
    ids = [f"{UUIDS[i]}_1" for i in range(3)]
    seq = [("R", AddMessage(UUIDS[0], 1, paths[0], 0)), ("R", AddMessage(UUIDS[1], 1, paths[1], 0)),
           ("R", AddMessage(UUIDS[2], 1, str(narrow), 0)),
           ("L", RecordBatch(X, model_ids=np.array(ids, dtype=object)[code]))]
    env = StreamExecutionEnvironment()
    ev, ctrl = env.from_either(seq)
    (pb, _), = ev.with_support_stream(ctrl).quick_evaluate().collect()
    assert not pb.valid[code == 2].any()
    for i in range(2):
        rows = np.flatnonzero(code == i)
        ref = PmmlModel.from_path(paths[i]).predict(X[rows])
        assert (pb.valid[rows] == ref.valid).all() and ref.valid.any()


def test_dynamic_quick_evaluate_per_record_events(tmp_path):
    from tests.test_stream import DynamicInput

    paths = _models(tmp_path, k=1, n_features=4)
    ev = [DynamicInput(f"{UUIDS[0]}_1", (1.0, 2.0, 3.0, 4.0), occurred_on=i) for i in range(3)]
    env = StreamExecutionEnvironment()
    events, ctrl = env.from_either([("R", AddMessage(UUIDS[0], 1, paths[0], 0))] + [("L", e) for e in ev])
    out = events.with_support_stream(ctrl).quick_evaluate().collect()
    ref = PmmlModel.from_path(paths[0]).predict(ev[0].to_vector())
    assert [p for p, _ in out] == [ref] * 3 and [e for _, e in out] == ev


# ----------------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("n_models", [3, 64, 300])
def test_grouped_device_pass_matches_oracle(gpu, tmp_path, n_models):
    """The grouped pass (one H2D, group_rows_kernel, one launch per model, ungroup_kernel) on
    uint8 / int16 codes: every model's rows equal that model's fp64 oracle."""
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.utils.metrics import METRICS

    F = 16
    kinds = max(1, min(n_models, 6))
    docs = [synth.gbdt_pmml(n_trees=20 + 7 * i, depth=3 + i % 4, n_features=F, seed=i) if i % 3 else
            synth.random_forest_pmml(n_trees=8, depth=5, n_features=F, n_classes=3, seed=i) for i in range(kinds)]
    paths = []
    for i, d in enumerate(docs):
        p = tmp_path / f"k{i}.pmml"
        p.write_text(d)
        paths.append(str(p))
    uuids = [f"a1b2c3d4-0000-4000-8000-{k:012d}" for k in range(n_models)]
    rng = np.random.default_rng(n_models)
    n = 300_000
    X = synth.stream_matrix(n, F, seed=5, missing_rate=0.02).astype(np.float32)
    code = rng.integers(0, n_models + 1, n)  # the last code: an unknown id (EmptyScore)
    ids = [f"{u}_1" for u in uuids] + ["ffffffff-0000-4000-8000-000000000000_1"]
    seq = [("R", AddMessage(uuids[i], 1, paths[i % kinds], 0)) for i in range(n_models)]
    seq += [("L", RecordBatch(X, model_ids=(code, ids)))]
    cfg = ScoringConfig(device=gpu, fallback="error", micro_batch=1 << 17)
    before = METRICS.counters.get("grouped.batches", 0)
    env = StreamExecutionEnvironment(config=cfg)
    ev, ctrl = env.from_either(seq)
    (pb, _), = ev.with_support_stream(ctrl).quick_evaluate(config=cfg).collect()
    assert METRICS.counters.get("grouped.batches", 0) == before + 1  # the grouped device pass ran
    oracles = [CompiledPmml.from_string(d) for d in docs]
    for i in range(n_models + 1):
        rows = np.flatnonzero(code == i)
        if i == n_models:
            assert not pb.valid[rows].any()
            continue
        ref, vref = oracles[i % kinds].score_matrix_oracle(X[rows])
        assert (pb.valid[rows] == vref).all(), i
        np.testing.assert_allclose(pb.scores[rows][vref], ref[vref], atol=2e-5, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n_models", [5, 64])
def test_device_counted_grouped_pass(gpu, tmp_path, n_models):
    """when every served model scores with the wide tree kernel the grouped pass
    counts on the device and issues ONE tree launch per kernel configuration per slice (here:
    depths 4 / 6 / 7 GBDTs + a fp32 random forest vote -> a handful of launches, not one per
    model). Every model's rows equal its fp64 oracle; unknown ids are EmptyScore."""
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.utils.metrics import METRICS

    F = 16
    docs = [synth.gbdt_pmml(n_trees=80, depth=6, n_features=F, seed=1),
            synth.gbdt_pmml(n_trees=96, depth=4, n_features=F, seed=2),
            synth.gbdt_pmml(n_trees=64, depth=7, n_features=F, seed=3),
            synth.gbdt_pmml(n_trees=70, depth=6, n_features=F, seed=4, objective="binary"),
            synth.random_forest_pmml(n_trees=64, depth=6, n_features=F, n_classes=3, seed=5)]
    paths = []
    for i, d in enumerate(docs):
        p = tmp_path / f"d{i}.pmml"
        p.write_text(d)
        paths.append(str(p))
    uuids = [f"a1b2c3d4-0000-4000-8000-{k:012d}" for k in range(n_models)]
    rng = np.random.default_rng(7 + n_models)
    n = 700_001
    X = synth.stream_matrix(n, F, seed=8, missing_rate=0.03).astype(np.float32)
    code = rng.integers(0, n_models + 1, n)
    ids = [f"{u}_1" for u in uuids] + ["ffffffff-0000-4000-8000-000000000000_1"]
    seq = [("R", AddMessage(uuids[i], 1, paths[i % len(docs)], 0)) for i in range(n_models)]
    seq += [("L", RecordBatch(X, model_ids=(code, ids)))]
    cfg = ScoringConfig(device=gpu, fallback="error", micro_batch=1 << 17)
    before = METRICS.counters.get("grouped.device_counted_batches", 0)
    launches = METRICS.counters.get("grouped.tree_launches", 0)
    slices = METRICS.counters.get("grouped.slices", 0)
    env = StreamExecutionEnvironment(config=cfg)
    ev, ctrl = env.from_either(seq)
    (pb, _), = ev.with_support_stream(ctrl).quick_evaluate(config=cfg).collect()
    assert METRICS.counters.get("grouped.device_counted_batches", 0) == before + 1
    n_slices = METRICS.counters.get("grouped.slices", 0) - slices
    per_slice = (METRICS.counters.get("grouped.tree_launches", 0) - launches) / n_slices
    assert per_slice <= len(docs)  # one launch per kernel configuration, whatever n_models
    oracles = [CompiledPmml.from_string(d) for d in docs]
    for i in range(n_models + 1):
        rows = np.flatnonzero(code == i)
        if i == n_models:
            assert not pb.valid[rows].any()
            continue
        ref, vref = oracles[i % len(docs)].score_matrix_oracle(X[rows])
        assert (pb.valid[rows] == vref).all(), i
        np.testing.assert_allclose(pb.scores[rows][vref], ref[vref], atol=2e-5, rtol=0)


@pytest.mark.gpu
def test_device_tables_built_while_default_stream_busy(gpu, tmp_path):
    """the device-counted tables (zeroed ``counts`` / ``ticket``) must be ready
    on the compute stream even when the default stream is still busy when they are created."""
    import torch

    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.engine import DevicePipeline
    from flink_jpmml_amd.runtime.grouped import GroupedScorer
    from flink_jpmml_amd.runtime.loading import load_local

    F = 16
    docs = [synth.gbdt_pmml(n_trees=40, depth=6, n_features=F, seed=s) for s in (11, 12, 13)]
    cfg = ScoringConfig(device=gpu, fallback="error", micro_batch=1 << 16)
    pipe = DevicePipeline(gpu, micro_batch=1 << 16)
    models = []
    for i, d in enumerate(docs):
        p = tmp_path / f"s{i}.pmml"
        p.write_text(d)
        models.append(load_local(str(p), gpu, cfg, pipe).model)
    n = 200_003
    X = synth.stream_matrix(n, F, seed=3, missing_rate=0.02).astype(np.float32)
    code = np.random.default_rng(1).integers(0, 3, n).astype(np.uint8)
    gs = GroupedScorer(pipe)
    # poison the allocator's next int32 blocks, then keep the default stream busy while the tables
    # are created: a zero-fill enqueued there would land after the count kernel ran
    junk = torch.full((1 << 20,), 12345, dtype=torch.int32, device=gpu)
    del junk
    torch.cuda._sleep(200_000_000)
    pb = gs.submit(RecordBatch(X), torch.from_numpy(code).pin_memory(), [m.scorer for m in models])
    pb.wait()
    torch.cuda.synchronize()
    for k, d in enumerate(docs):
        rows = np.flatnonzero(code == k)
        ref, vref = CompiledPmml.from_string(d).score_matrix_oracle(X[rows])
        assert (pb.valid[rows] == vref).all(), k
        np.testing.assert_allclose(pb.scores[rows][vref], ref[vref], atol=2e-5, rtol=0)


@pytest.mark.gpu
def test_out_of_range_pinned_codes_raise_like_host_codes(gpu, tmp_path):
    """pinned codes outside [0, K) raise ValueError on the device-counted path too."""
    import torch

    from flink_jpmml_amd.runtime.engine import DevicePipeline
    from flink_jpmml_amd.runtime.grouped import GroupedScorer
    from flink_jpmml_amd.runtime.loading import load_local

    F = 8
    pipe = DevicePipeline(gpu, micro_batch=1 << 14)
    cfg = ScoringConfig(device=gpu, fallback="error", micro_batch=1 << 14)
    scorers = []
    for s in (1, 2):
        p = tmp_path / f"o{s}.pmml"
        p.write_text(synth.gbdt_pmml(n_trees=8, depth=4, n_features=F, seed=s))
        scorers.append(load_local(str(p), gpu, cfg, pipe).model.scorer)
    X = synth.stream_matrix(1000, F, seed=2).astype(np.float32)
    codes = torch.zeros(1000, dtype=torch.uint8).pin_memory()
    codes[17] = 5
    with pytest.raises(ValueError):
        GroupedScorer(pipe).submit(RecordBatch(X), codes, scorers)
    with pytest.raises(ValueError):
        GroupedScorer(pipe).submit(RecordBatch(X), codes.numpy().copy(), scorers)
