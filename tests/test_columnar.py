"""Columnar (RecordBatch) DSL path, lazy PredictionBatch, latency-bound micro-batches, replay
verification and replace_nan parity — on the host scorer (the GPU variants live in
test_gpu_dsl.py). Every batched result is compared with the reference's per-record contract."""

import numpy as np
import pytest

from flink_jpmml_amd import AddMessage, DelMessage, DenseVector, ModelReader, SparseVector
from flink_jpmml_amd.api.batch import PredictionBatch, RecordBatch
from flink_jpmml_amd.api.exceptions import NoSuchElementException
from flink_jpmml_amd.api.pmml_model import PmmlModel
from flink_jpmml_amd.config import ScoringConfig
from flink_jpmml_amd.domain import EmptyScore, Prediction, Score
from flink_jpmml_amd.stream import ManualClock, StreamExecutionEnvironment
from flink_jpmml_amd.stream.clock import current_clock
from flink_jpmml_amd.utils.metrics import METRICS

N1 = "a1b2c3d4-0000-4000-8000-000000000001"
N2 = "a1b2c3d4-0000-4000-8000-000000000002"


def _matrix(n, seed=0, missing=0.0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0.2, 7.0, size=(n, 4))
    if missing:
        X[rng.random(X.shape) < missing] = np.nan
    return X


def test_prediction_batch_matches_per_record_predict(fixtures_dir):
    model = PmmlModel.from_path(fixtures_dir["kmeans"])
    X = _matrix(200, missing=0.1)
    pb = model.predict(RecordBatch(X))
    assert isinstance(pb, PredictionBatch) and len(pb) == 200
    per_record = [model.predict(DenseVector(row)) for row in X]
    assert pb.to_list() == per_record
    assert pb[3] == per_record[3] and list(pb)[:5] == per_record[:5]
    assert np.array_equal(pb.values(-1.0), [p.value.get_or_else(-1.0) for p in per_record])
    # a 2-D array is a batch too; a wrong width is EmptyScore for every row (validation)
    assert model.predict(X[:3]).to_list() == per_record[:3]
    assert model.predict(RecordBatch(X[:, :3])).to_list() == [Prediction(EmptyScore)] * 200


def test_from_vectors_keeps_sparse_absent_semantics(fixtures_dir):
    """replace_nan fills only entries a sparse vector does not store; a NaN stored in a
    dense vector stays a PMML missing value — batched == per record."""
    model = PmmlModel.from_path(fixtures_dir["kmeans"])
    vecs = [DenseVector(1.0, float("nan"), 1.0, 1.0), SparseVector(4, [0, 2], [1.0, 2.0]),
            DenseVector(6.0, float("nan"), 5.0, 2.0), SparseVector(4, [1, 3], [3.0, float("nan")]), DenseVector(1, 2)]
    for rn in (None, 0.0, 9.0):
        per_record = [model.predict(v, rn) for v in vecs]
        batched = model.predict_records(RecordBatch.from_vectors(vecs, 4), rn).to_list()
        assert batched == per_record, rn
        assert model.predict_vectors(vecs, replace_nan=rn) == per_record


def test_quick_evaluate_columnar(fixtures_dir):
    X = _matrix(1000, seed=1, missing=0.05)
    env = StreamExecutionEnvironment()
    out = env.from_batches(X, batch_rows=128).quick_evaluate(ModelReader(fixtures_dir["kmeans"])).collect()
    assert len(out) == 8 and all(isinstance(p, PredictionBatch) and isinstance(b, RecordBatch) for p, b in out)
    model = PmmlModel.from_path(fixtures_dir["kmeans"])
    got = [p for pb, _ in out for p in pb]
    assert got == [model.predict(DenseVector(r)) for r in X]
    # unbatch() turns them into the reference's (Prediction, vector) elements
    env2 = StreamExecutionEnvironment()
    flat = env2.from_batches(X[:10], batch_rows=4).quick_evaluate(ModelReader(fixtures_dir["kmeans"])).unbatch() \
        .collect()
    assert [p for p, _ in flat] == got[:10] and flat[0][1] == DenseVector(X[0])


def test_evaluate_columnar_udf_gets_whole_batch(fixtures_dir):
    X = _matrix(300, seed=2)
    env = StreamExecutionEnvironment()
    out = env.from_batches(X, batch_rows=100).evaluate(
        ModelReader(fixtures_dir["kmeans"]), lambda b, m: (b.offset, m.predict(b).values(-1.0))).collect()
    assert [o for o, _ in out] == [0, 100, 200]
    model = PmmlModel.from_path(fixtures_dir["kmeans"])
    np.testing.assert_array_equal(np.concatenate([v for _, v in out]), model.predict(X).values(-1.0))


def test_dynamic_columnar_single_and_mixed_ids(fixtures_dir):
    X = _matrix(40, seed=3)
    ids = np.array([f"{N1}_1" if i % 3 else f"{N2}_1" for i in range(40)], dtype=object)
    seq = [("L", RecordBatch(X[:10], model_id=f"{N1}_1")),
           ("R", AddMessage(N1, 1, fixtures_dir["kmeans"], 0)),
           ("L", RecordBatch(X[:10], model_id=f"{N1}_1")),
           ("L", RecordBatch(X, model_ids=ids)),
           ("R", DelMessage(N1, 1, 0)),
           ("L", RecordBatch(X[:5], model_id=f"{N1}_1"))]
    env = StreamExecutionEnvironment()
    ev, ctrl = env.from_either(seq)
    out = ev.with_support_stream(ctrl).evaluate(lambda b, m: (b.model_id, b.row_index, m.predict(b))).collect()
    model = PmmlModel.from_path(fixtures_dir["kmeans"])
    ref = model.predict(X).to_list()
    assert out[0][2].to_list() == [Prediction(EmptyScore)] * 10  # before Add
    assert out[1][2].to_list() == ref[:10]
    # the mixed batch is split per model id (first appearance order), row_index maps back
    (mid_a, rows_a, pa), (mid_b, rows_b, pb) = out[2], out[3]
    assert mid_a == f"{N2}_1" and mid_b == f"{N1}_1"
    assert pa.to_list() == [Prediction(EmptyScore)] * len(rows_a)  # N2 never added
    assert pb.to_list() == [ref[i] for i in rows_b]
    assert sorted(np.concatenate([rows_a, rows_b]).tolist()) == list(range(40))
    assert out[4][2].to_list() == [Prediction(EmptyScore)] * 5  # after Del


# ------------------------------------------------------------------ latency-bound micro-batches


class SlowSource:
    """1 record / virtual second (the reference's IrisSource rate, `E/sources/IrisSource.scala:52`)."""

    def __init__(self, n, log):
        self.n = n
        self.log = log

    def __iter__(self):
        clock = current_clock()
        for i in range(self.n):
            clock.sleep(1.0)
            self.log.append((i, clock.now()))
            yield DenseVector(1.0 + i % 3, 1.0, 1.0, 1.0)


@pytest.mark.parametrize("api", ["quick", "evaluate"])
def test_latency_trigger_flushes_slow_stream(fixtures_dir, api):
    clock = ManualClock()
    arrivals, emitted = [], []
    env = StreamExecutionEnvironment(clock=clock)
    src = env.add_source(_IterSource(SlowSource(6, arrivals)))
    cfg = ScoringConfig(batch_size=65536, max_batch_latency_ms=100.0)
    if api == "quick":
        s = src.quick_evaluate(ModelReader(fixtures_dir["kmeans"]), config=cfg)
    else:
        s = src.evaluate(ModelReader(fixtures_dir["kmeans"]), lambda v, m: (v, m.predict(v)), config=cfg)
    s.add_sink(lambda x: emitted.append(clock.now()))
    env.execute()
    assert len(emitted) == 6
    for (i, t_in), t_out in zip(arrivals[:-1], emitted):
        assert t_out - t_in == pytest.approx(0.1), (i, t_in, t_out)  # emitted at the bound, not at the end
    assert emitted[-1] == arrivals[-1][1]  # the last one is flushed by the end of input


def test_no_latency_bound_waits_for_size_or_end(fixtures_dir):
    clock = ManualClock()
    arrivals, emitted = [], []
    env = StreamExecutionEnvironment(clock=clock)
    env.add_source(_IterSource(SlowSource(5, arrivals))).quick_evaluate(
        ModelReader(fixtures_dir["kmeans"]), batch_size=65536).add_sink(lambda x: emitted.append(clock.now()))
    env.execute()
    assert emitted == [5.0] * 5  # everything at end of input


class _IterSource:
    def __init__(self, it):
        self.it = it

    def __iter__(self):
        return iter(self.it)


# ------------------------------------------------------------------ replay verification


def test_udf_branching_on_score_is_batch_invariant(fixtures_dir):
    vals = [(1.0, 1.0, 1.0, 1.0), (1.0, 2.0, 3.0, 4.0), (6.9, 3.1, 5.8, 2.1), (5.0, 3.0, 1.5, 0.2)] * 4

    def udf(e, m):
        p = m.predict(DenseVector(*e))
        if p.value.get_or_else(-1.0) >= 3.0:  # a second predict only on some scores
            q = m.predict(DenseVector(*[x + 1 for x in e]))
            return ("hi", p, q)
        return ("lo", p)

    ref = StreamExecutionEnvironment().from_collection(vals).evaluate(ModelReader(fixtures_dir["kmeans"]), udf).collect()
    out = StreamExecutionEnvironment().from_collection(vals).evaluate(
        ModelReader(fixtures_dir["kmeans"]), udf, batch_size=5).collect()
    assert out == ref  # deferred mode: the branch resolves the pending calls, f runs once
    before = METRICS.counters.get("batcher.per_record_reruns", 0)
    out = StreamExecutionEnvironment().from_collection(vals).evaluate(
        ModelReader(fixtures_dir["kmeans"]), udf, config=ScoringConfig(batch_size=5, udf_mode="replay")).collect()
    assert out == ref
    assert METRICS.counters.get("batcher.per_record_reruns", 0) > before


def test_udf_calling_get_is_batch_invariant(fixtures_dir):
    vals = [(1.0, 1.0, 1.0, 1.0), (1.0, 2.0), (6.9, 3.1, 5.8, 2.1)]

    def udf(e, m):
        try:
            return m.predict(DenseVector(*e)).value.get()
        except NoSuchElementException:
            return "empty"

    ref = StreamExecutionEnvironment().from_collection(vals).evaluate(ModelReader(fixtures_dir["kmeans"]), udf).collect()
    out = StreamExecutionEnvironment().from_collection(vals).evaluate(
        ModelReader(fixtures_dir["kmeans"]), udf, batch_size=8).collect()
    assert out == ref and ref[1] == "empty" and isinstance(ref[0], float)

    def strict(e, m):  # .get() raising inside the UDF: the capture pass fails -> per-record rerun
        return m.predict(DenseVector(*e)).value.get()

    out2 = StreamExecutionEnvironment().from_collection([vals[0], vals[2]]).evaluate(
        ModelReader(fixtures_dir["kmeans"]), strict, batch_size=8).collect()
    assert out2 == [ref[0], ref[2]]


# ------------------------------------------------------------------ config


def test_scoring_config_validation_and_env(monkeypatch):
    with pytest.raises(ValueError):
        ScoringConfig(precision="fp16")
    with pytest.raises(ValueError):
        ScoringConfig(fallback="maybe")
    monkeypatch.setenv("FJA_BATCH_SIZE", "4096")
    monkeypatch.setenv("FJA_MAX_BATCH_LATENCY_MS", "2.5")
    monkeypatch.setenv("FJA_PRECISION", "fp8")
    cfg = ScoringConfig.from_env()
    assert cfg.batch_size == 4096 and cfg.max_batch_latency_ms == 2.5 and cfg.precision == "fp8"
    assert cfg.lowering_opts() == {"precision": "fp8"}
    assert ScoringConfig(device=None).resolve_device() is None


def test_host_fallback_policy_counts_and_can_refuse(fixtures_dir, monkeypatch):
    """A model the device cannot lower is never silently demoted: fallback='error' refuses it."""
    from flink_jpmml_amd.api.exceptions import ModelLoadingException
    from flink_jpmml_amd.runtime import engine
    from flink_jpmml_amd.runtime.plans import NotLowerable

    model = PmmlModel.from_path(fixtures_dir["kmeans"])

    def boom(*a, **k):
        raise NotLowerable("test: not lowerable")

    monkeypatch.setattr(type(model.compiled), "plan", boom)
    before = METRICS.counters.get("scoring.host_fallback_models", 0)
    sc = engine.make_scorer(model.compiled, "cuda:0", ScoringConfig(fallback="warn"))
    assert sc.kind == "host" and METRICS.counters["scoring.host_fallback_models"] == before + 1
    with pytest.raises(ModelLoadingException):
        engine.make_scorer(model.compiled, "cuda:0", ScoringConfig(fallback="error"))
    X = _matrix(7, seed=9)
    assert sc.submit_batch(RecordBatch(X)).to_list() == [model.predict(DenseVector(r)) for r in X]


def test_dense_nan_is_not_replaced_in_batches(fixtures_dir):
    """A NaN *stored* in a DenseVector stays a PMML missing value under replace_nan (the key is
    present in the reference's input map, `S/api/PmmlModel.scala:143-152`): batched == per record."""
    from flink_jpmml_amd.api.pmml_model import PmmlModel

    m = PmmlModel.from_path(fixtures_dir["kmeans"])
    vecs = [DenseVector(1.0, float("nan"), 1.0, 1.0), DenseVector(6.9, 3.1, 5.8, 2.1)]
    per = [m.predict(v, 0.0) for v in vecs]
    batch = RecordBatch.from_vectors(vecs, 4)
    assert m.predict_records(batch, replace_nan=0.0).to_list() == per
    assert m.predict_vectors(vecs, replace_nan=0.0) == per


@pytest.mark.parametrize("chunked", [True, False])
def test_batched_udf_runs_exactly_once_per_event(fixtures_dir, chunked):
    """with batch_size set the UDF is called once per event (side effects
    once), its predictions are scored in one batch per flush, results equal per-record."""
    calls = []
    vals = [(1.0, 1.0, 1.0, 1.0), (1.0, 2.0, 3.0, 4.0), (1.0, 2.0), (6.9, 3.1, 5.8, 2.1)] * 25

    def udf(e, m):
        calls.append(e)
        return e, m.predict(DenseVector(*e))

    ref = StreamExecutionEnvironment().from_collection(vals).evaluate(
        ModelReader(fixtures_dir["kmeans"]), lambda e, m: (e, m.predict(DenseVector(*e)))).collect()
    env = StreamExecutionEnvironment()
    src = env.from_collection(vals) if chunked else env.add_source(_IterSource(vals))
    before = METRICS.counters.get("batcher.resolves", 0)
    out = src.evaluate(ModelReader(fixtures_dir["kmeans"]), udf, batch_size=16).collect()
    assert len(calls) == len(vals)  # exactly once per event
    assert out == ref
    assert METRICS.counters.get("batcher.resolves", 0) - before == -(-len(vals) // 16)  # one per batch


def test_dynamic_batched_udf_exactly_once_with_lazy_value(fixtures_dir):
    """The reference's dynamic UDF returns ``prediction.value`` (E/DynamicEvaluateKmeans.scala:54-60):
    reading ``.value`` resolves the pending calls (the UDF sees a real Target), the UDF still runs
    exactly once per event, and Add/Del boundaries keep their semantics."""
    seen = []
    seq = [("L", (N1, (1.0, 1.0, 1.0, 1.0))), ("R", AddMessage(N1, 1, fixtures_dir["kmeans"], 0))] + \
          [("L", (N1, (1.0 + i / 10, 2.0, 3.0, 1.0))) for i in range(20)] + [("R", DelMessage(N1, 1, 0))] + \
          [("L", (N1, (1.0, 1.0, 1.0, 1.0)))]

    class Ev:
        def __init__(self, mid, v):
            self.model_id, self.v = f"{mid}_1", v

    def udf(e, m):
        seen.append(e)
        return m.predict(DenseVector(*e.v), 0.0).value

    def run(bs):
        env = StreamExecutionEnvironment()
        ev, ctrl = env.from_either([(t, Ev(*x) if t == "L" else x) for t, x in seq])
        return ev.with_support_stream(ctrl).evaluate(udf, batch_size=bs).collect()

    ref = run(None)
    n = len(seen)
    out = run(8)
    assert len(seen) == 2 * n  # once per event in each run
    assert [repr(t) for t in out] == [repr(t) for t in ref]
    assert repr(out[0]) == "EmptyScore" and repr(out[-1]) == "EmptyScore" and out[1] == Score(3.0)


@pytest.mark.parametrize("bs", [None, 8])
def test_batched_udf_sees_real_score_and_empty_score(fixtures_dir, bs):
    """under ``batch_size`` a UDF that pattern-matches the Target inside ``f`` (the
    reference's ``case Score(v) / case EmptyScore``) gets the real objects, not a lazy stand-in."""
    from flink_jpmml_amd.domain import EmptyScore as EMPTY

    vals = [(1.0, 1.0, 1.0, 1.0), (1.0, 2.0), (6.9, 3.1, 5.8, 2.1), (1.0,)] * 6

    def udf(e, m):
        p = m.predict(DenseVector(*e))
        t = p.value
        if isinstance(t, Score):
            return ("score", t.value)
        if t is EMPTY:
            return ("empty", None)
        return ("neither", repr(t))

    env = StreamExecutionEnvironment()
    out = env.from_collection(vals).evaluate(ModelReader(fixtures_dir["kmeans"]), udf, batch_size=bs).collect()
    assert [k for k, _ in out] == ["score", "empty", "score", "empty"] * 6
    assert out[0] == ("score", 3.0)


def test_to_batches_adapter_matches_per_record(fixtures_dir):
    """events.to_batches(extract) → RecordBatches → quick_evaluate → unbatch gives each event's
    per-record prediction (vectorised event → RecordBatch adapter)."""
    from tests.test_stream import DynamicInput

    m = PmmlModel.from_path(fixtures_dir["kmeans"])
    evs = [DynamicInput(f"{N1}_1", (1.0 + (i % 9) / 2, 2.0, 3.0 - (i % 4) / 3, 1.0), occurred_on=i) for i in range(700)]
    env = StreamExecutionEnvironment()
    out = env.from_collection(evs).to_batches(lambda e: e.values, batch_rows=128) \
        .quick_evaluate(ModelReader(fixtures_dir["kmeans"])).unbatch().collect()
    assert [e for _, e in out] == evs
    assert [p for p, _ in out] == [m.predict(e.to_vector()) for e in evs]


def test_to_batches_dynamic_ids_and_latency(fixtures_dir):
    seq = [("R", AddMessage(N1, 1, fixtures_dir["kmeans"], 0))] + \
          [("L", (f"{N1 if i % 2 else N2}_1", (1.0, 1.0, 1.0, 1.0))) for i in range(10)]
    env = StreamExecutionEnvironment()
    ev, ctrl = env.from_either(seq)
    batches = ev.to_batches(lambda e: e[1], batch_rows=4, model_id=lambda e: e[0])
    out = batches.with_support_stream(ctrl).evaluate(lambda b, m: (b.model_id, m.predict(b).values(-1.0).tolist())) \
        .collect()
    got = {}
    for mid, vals in out:
        got.setdefault(mid, []).extend(vals)
    assert got[f"{N1}_1"] == [3.0] * 5 and got[f"{N2}_1"] == [-1.0] * 5


def test_device_auto_is_the_default_and_resolves_to_the_host_without_a_gpu():
    import torch

    cfg = ScoringConfig()
    assert cfg.device == "auto"
    if not torch.cuda.is_available():
        assert cfg.resolve_device() is None
    assert ScoringConfig(device="cpu").resolve_device() is None
    assert ScoringConfig(device=None).resolve_device() is None
