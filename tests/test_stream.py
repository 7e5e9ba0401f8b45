"""Ports of the reference's integration specs on the mini stream runtime:
RichDataStreamSpec, QuickDataStreamSpec, EvaluationFunctionSpec, EvaluationCoFunctionSpec and the
15 RichConnectedStreamSpec scenarios, plus checkpoint/restore (untested in the reference)."""

import uuid
from dataclasses import dataclass

import pytest

from flink_jpmml_amd import AddMessage, DelMessage, DenseVector, ModelReader, SparseVector
from flink_jpmml_amd.api.exceptions import ModelLoadingException, WrongModelIdFormat
from flink_jpmml_amd.domain import EmptyScore, Prediction, Score
from flink_jpmml_amd.stream import (
    EvaluationCoFunction,
    EvaluationFunction,
    JobExecutionException,
    SimulatedFailure,
    StreamExecutionEnvironment,
    ensure_serializable,
)


@dataclass(frozen=True)
class Input:
    values: tuple

    def to_vector(self):
        return DenseVector(*self.values)


@dataclass(frozen=True)
class DynamicInput:
    model_id: str
    values: tuple
    occurred_on: int = 0

    def to_vector(self):
        return DenseVector(*self.values)


ONES = (1.0, 1.0, 1.0, 1.0)
N1 = "a1b2c3d4-0000-4000-8000-000000000001"
N2 = "a1b2c3d4-0000-4000-8000-000000000002"


def udf(event, model):
    return model.predict(event.to_vector(), None)


# ------------------------------------------------------------------ RichDataStreamSpec (:65-107)
def test_evaluate_is_serializable(fixtures_dir):
    op = EvaluationFunction(ModelReader(fixtures_dir["kmeans"]), udf)
    ensure_serializable(op)


def test_evaluate_golden(fixtures_dir):
    env = StreamExecutionEnvironment()
    out = env.from_collection([Input(ONES)]).evaluate(ModelReader(fixtures_dir["kmeans"]), udf).collect()
    assert out == [Prediction(Score(3.0))]


def test_evaluate_missing_model_path_fails_job(tmp_path):
    env = StreamExecutionEnvironment()
    s = env.from_collection([Input(ONES)]).evaluate(ModelReader(str(tmp_path / "nope.xml")), udf)
    with pytest.raises(JobExecutionException) as ei:
        s.collect()
    assert isinstance(ei.value.__cause__, ModelLoadingException)


def test_evaluate_bad_input_is_empty(fixtures_dir):
    env = StreamExecutionEnvironment()
    out = env.from_collection([Input((1.0, 2.0))]).evaluate(ModelReader(fixtures_dir["kmeans"]), udf).collect()
    assert out == [Prediction(EmptyScore)]


def test_evaluate_empty_pmml_fails_job(fixtures_dir):
    env = StreamExecutionEnvironment()
    s = env.from_collection([Input(ONES)]).evaluate(ModelReader(fixtures_dir["kmeans_empty"]), udf)
    with pytest.raises(JobExecutionException):
        s.collect()


# ------------------------------------------------------------------ QuickDataStreamSpec (:56-104)
@pytest.mark.parametrize("batch", [None, 2, 64])
def test_quick_evaluate_dense_and_sparse(fixtures_dir, batch):
    env = StreamExecutionEnvironment()
    vecs = [DenseVector(*ONES), SparseVector(4, [0, 1, 2, 3], [1.0] * 4), DenseVector(*ONES)]
    out = env.from_collection(vecs).quick_evaluate(ModelReader(fixtures_dir["kmeans"]), batch_size=batch).collect()
    assert out == [(Prediction(Score(3.0)), v) for v in vecs]


def test_quick_evaluate_short_sparse_is_empty(fixtures_dir):
    env = StreamExecutionEnvironment()
    v = SparseVector(2, [0], [1.0])
    out = env.from_collection([v]).quick_evaluate(ModelReader(fixtures_dir["kmeans"]), batch_size=4).collect()
    assert out == [(Prediction(EmptyScore), v)]


@pytest.mark.parametrize("name", ["kmeans_empty", "missing"])
def test_quick_evaluate_load_failures(fixtures_dir, tmp_path, name):
    path = fixtures_dir.get(name, str(tmp_path / "missing.xml"))
    env = StreamExecutionEnvironment()
    with pytest.raises(JobExecutionException):
        env.from_collection([DenseVector(*ONES)]).quick_evaluate(ModelReader(path)).collect()


# ------------------------------------------------------------------ EvaluationFunctionSpec
def test_evaluation_function_emits_udf_result(fixtures_dir):
    env = StreamExecutionEnvironment()
    out = env.from_collection([Input(ONES)]).evaluate(
        ModelReader(fixtures_dir["kmeans"]), lambda e, m: m.predict(e.to_vector()).value.get_or_else(-1.0)).collect()
    assert out == [3.0]


# ------------------------------------------------------------------ EvaluationCoFunctionSpec (:81-146)
def test_co_function_load_and_metadata(fixtures_dir):
    op = EvaluationCoFunction(udf)
    ensure_serializable(op)
    assert op.load_model(fixtures_dir["kmeans"]).model_name == "k-means"
    with pytest.raises(ModelLoadingException):
        op.load_model(fixtures_dir["kmeans_empty"])
    assert op.from_metadata(f"{N1}_1").is_empty
    for bad in ["abc_1", f"{N1}", "x"]:
        with pytest.raises(WrongModelIdFormat):
            op.from_metadata(bad)


# ------------------------------------------------------------------ RichConnectedStreamSpec (:69-337)
def add(name, version, path):
    return ("R", AddMessage(name, version, path, 0))


def dele(name, version):
    return ("R", DelMessage(name, version, 0))


def ev(name, version, values=ONES):
    return ("L", DynamicInput(f"{name}_{version}", values))


def run_dynamic(seq, batch=None, parallelism=1, f=udf):
    env = StreamExecutionEnvironment(parallelism)
    events, control = env.from_either(seq)
    return events.with_support_stream(control).evaluate(f, batch_size=batch).collect()


S3 = Prediction(Score(3.0))
E = Prediction(EmptyScore)
BATCHES = [None, 1, 3, 100]


@pytest.mark.parametrize("batch", BATCHES)
def test_model_then_event(fixtures_dir, batch):
    assert run_dynamic([add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1)], batch) == [S3]


@pytest.mark.parametrize("batch", BATCHES)
def test_event_model_event(fixtures_dir, batch):
    assert run_dynamic([ev(N1, 1), add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1)], batch) == [E, S3]


@pytest.mark.parametrize("batch", BATCHES)
def test_two_models_one_without_target(fixtures_dir, batch):
    seq = [add(N1, 1, fixtures_dir["kmeans"]), add(N2, 1, fixtures_dir["kmeans_nooutput_notarget"]),
           ev(N1, 1), ev(N2, 1)]
    assert run_dynamic(seq, batch) == [S3, E]


@pytest.mark.parametrize("batch", BATCHES)
def test_interleaved(fixtures_dir, batch):
    seq = [ev(N1, 1), add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), ev(N2, 1),
           add(N2, 1, fixtures_dir["kmeans_nooutput"]), ev(N2, 1), ev(N1, 1)]
    assert run_dynamic(seq, batch) == [E, S3, E, S3, S3]


def test_only_events(fixtures_dir):
    assert run_dynamic([ev(N1, 1), ev(N2, 3)]) == [E, E]


def test_only_models(fixtures_dir):
    assert run_dynamic([add(N1, 1, fixtures_dir["kmeans"]), add(N2, 1, fixtures_dir["kmeans"])]) == []


def test_del_without_model(fixtures_dir):
    assert run_dynamic([dele(N1, 1), ev(N1, 1)]) == [E]


@pytest.mark.parametrize("batch", BATCHES)
def test_del_current_model_evicts(fixtures_dir, batch):
    seq = [add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), dele(N1, 1), ev(N1, 1)]
    assert run_dynamic(seq, batch) == [S3, E]


def test_del_other_model_no_effect(fixtures_dir):
    seq = [add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), dele(N2, 1), ev(N1, 1)]
    assert run_dynamic(seq) == [S3, S3]


@pytest.mark.parametrize("batch", BATCHES)
def test_add_del_add(fixtures_dir, batch):
    seq = [add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), dele(N1, 1), ev(N1, 1),
           add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1)]
    assert run_dynamic(seq, batch) == [S3, E, S3]


def test_del_add_del(fixtures_dir):
    seq = [dele(N1, 1), ev(N1, 1), add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), dele(N1, 1), ev(N1, 1)]
    assert run_dynamic(seq) == [E, S3, E]


def test_duplicate_add_is_ignored(fixtures_dir):
    # second Add with the same id points at a no-target model: ignored -> still Score(3.0)
    seq = [add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1), add(N1, 1, fixtures_dir["kmeans_nooutput_notarget"]),
           ev(N1, 1)]
    assert run_dynamic(seq) == [S3, S3]


def test_bad_path_fails_job(tmp_path):
    with pytest.raises(JobExecutionException):
        run_dynamic([add(N1, 1, str(tmp_path / "no.xml")), ev(N1, 1)])


def test_invalid_input_is_empty(fixtures_dir):
    seq = [add(N1, 1, fixtures_dir["kmeans"]), ev(N1, 1, (1.0, 2.0))]
    assert run_dynamic(seq) == [E]


def test_empty_pmml_fails_job(fixtures_dir):
    with pytest.raises(JobExecutionException):
        run_dynamic([add(N1, 1, fixtures_dir["kmeans_empty"]), ev(N1, 1)])


def test_wrong_model_id_fails_job(fixtures_dir):
    with pytest.raises(JobExecutionException) as ei:
        run_dynamic([("L", DynamicInput("not-an-id", ONES))])
    assert isinstance(ei.value.__cause__, WrongModelIdFormat)


@pytest.mark.parametrize("parallelism", [2, 3])
def test_parallel_subtasks_with_broadcast_control(fixtures_dir, parallelism):
    """Broadcast semantics with > 1 subtask (never exercised by the reference)."""
    seq = [add(N1, 1, fixtures_dir["kmeans"])] + [ev(N1, 1) for _ in range(7)] + [dele(N1, 1), ev(N1, 1)]
    out = run_dynamic(seq, parallelism=parallelism)
    assert sorted(out, key=repr) == sorted([S3] * 7 + [E], key=repr)


# ------------------------------------------------------------------ checkpoint / restore
def test_checkpoint_restore_metadata_only(fixtures_dir, tmp_path):
    env = StreamExecutionEnvironment(2)
    env.enable_checkpointing(every_n_records=2, directory=str(tmp_path))
    env.inject_failure(after_records=4)
    seq = [add(N1, 1, fixtures_dir["kmeans"]), add(N2, 1, fixtures_dir["kmeans"]), ev(N1, 1), ev(N2, 1),
           ev(N1, 1), ev(N2, 1)]
    events, control = env.from_either(seq)
    stream = events.with_support_stream(control).evaluate(udf, uid="scorer")
    with pytest.raises(JobExecutionException) as ei:
        stream.collect()
    assert isinstance(ei.value.__cause__, SimulatedFailure)
    latest = env.checkpoint_storage.latest()
    assert latest is not None
    # restart from the checkpoint with a NEW source (different uid: no offset to resume) holding
    # only events: the metadata (not the models) was restored
    env2 = StreamExecutionEnvironment(3)
    ev2, ctrl2 = env2.from_either([ev(N1, 1), ev(N2, 1), ev(N2, 7)], uid="fresh-source")
    out = ev2.with_support_stream(ctrl2).evaluate(udf, uid="scorer").collect(restore=latest)
    assert out == [S3, S3, E]
    doc = env.checkpoint_storage.read(latest)
    ops = doc["operators"]["scorer"]["metadata-snapshot"]
    assert ops["mode"] == "union" and len(ops["subtasks"]) == 2


def test_batched_udf_replays_in_order(fixtures_dir):
    """Micro-batched evaluate(): capture -> batch score -> replay keeps per-record semantics."""
    vals = [ONES, (1.0, 2.0, 3.0, 4.0), (1.0, 2.0), (6.9, 3.1, 5.8, 2.1)] * 5
    env = StreamExecutionEnvironment()
    out = env.from_collection([Input(v) for v in vals]).evaluate(
        ModelReader(fixtures_dir["kmeans"]), lambda e, m: (e.values, m.predict(e.to_vector()).value.get_or_else(-1.0)),
        batch_size=7).collect()
    env2 = StreamExecutionEnvironment()
    ref = env2.from_collection([Input(v) for v in vals]).evaluate(
        ModelReader(fixtures_dir["kmeans"]), lambda e, m: (e.values, m.predict(e.to_vector()).value.get_or_else(-1.0))
    ).collect()
    assert out == ref and out[0] == (ONES, 3.0) and out[2] == ((1.0, 2.0), -1.0)


def test_restore_resumes_source_offsets_exactly_once(fixtures_dir, tmp_path):
    """Same job restarted from its last checkpoint: the source resumes at the manifest's offset and
    a transactional FileSink commits per checkpoint, so both runs' committed outputs together
    equal one uninterrupted run (no duplicates, no gaps)."""
    from flink_jpmml_amd.stream import FileSink

    seq = [add(N1, 1, fixtures_dir["kmeans"])] + [ev(N1, 1, (1.0 + i / 10, 1.0, 1.0, 1.0)) for i in range(9)] + \
          [add(N2, 1, fixtures_dir["kmeans"])] + [ev(N2, 1, (5.0, 3.0, 5.0 + i / 10, 2.0)) for i in range(7)]

    def job(out_dir, ckpt_dir, fail_after=None, restore=None):
        env = StreamExecutionEnvironment()
        env.enable_checkpointing(every_n_records=4, directory=str(ckpt_dir))
        env.inject_failure(fail_after)
        events, control = env.from_either(seq)
        events.with_support_stream(control).evaluate(
            lambda e, m: [e.model_id, m.predict(e.to_vector()).value.get_or_else(-1.0)], uid="scorer"
        ).add_sink(FileSink(str(out_dir)))
        env.execute("exactly-once", restore=restore)
        return env

    ref_dir = tmp_path / "ref"
    job(ref_dir, tmp_path / "ck-ref")
    expected = FileSink.read(str(ref_dir))
    assert len(expected) == 16

    out_dir, ck = tmp_path / "out", tmp_path / "ck"
    with pytest.raises(JobExecutionException):
        job(out_dir, ck, fail_after=11)
    from flink_jpmml_amd.stream.state import CheckpointStorage

    latest = CheckpointStorage(str(ck)).latest()
    doc = CheckpointStorage.read(latest)
    assert doc["checkpoint_id"] == 2 and list(doc["sources"].values())[0]["offset"] == 8
    assert all(len(m["sha256"]) == 64 for m in doc["models"].values())
    assert len(FileSink.read(str(out_dir))) < len(expected)  # the crashed run committed a prefix
    job(out_dir, ck, restore=latest)
    assert FileSink.read(str(out_dir)) == expected
