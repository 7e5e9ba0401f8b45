"""Live streaming semantics of the runtime (VERDICT r2 "Next round" item 1): available-first input
multiplexing, live socket sources, time-based checkpoints, streaming sinks and exact offsets.

Reference behaviour: events keep flowing while the control stream is idle for seconds
(`E/CheckpointEvaluate.scala:56-82`: 1 Hz events + a socket control stream;
`E/DynamicEvaluateKmeans.scala:50-60` with control gaps up to 5000 ms,
`E/util/DynamicParams.scala:40`); checkpoints every ``interval`` ms (`E/DynamicEvaluateKmeans.scala:48`).
"""

import json
import os
import socket
import threading
import time

import pytest
import torch  # noqa: F401 - imported up front: a cold torch import inside a timed job is seconds

from flink_jpmml_amd import AddMessage, DelMessage, DenseVector
from flink_jpmml_amd.config import ScoringConfig
from flink_jpmml_amd.stream import FileSink, SourceFunction, StreamExecutionEnvironment
from flink_jpmml_amd.stream.state import CheckpointStorage
from tests.test_stream import N1, N2, DynamicInput


class PacedEvents(SourceFunction):
    """``n`` events every ``period_s`` (push source: runs on its own thread), stamping the wall
    clock at emission."""

    def __init__(self, n, period_s, model=N1, log=None):
        self.n = n
        self.period_s = period_s
        self.model = model
        self.log = log if log is not None else {}
        self._running = True

    def run(self, ctx):
        for i in range(self.n):
            if not self._running:
                return
            time.sleep(self.period_s)
            self.log[i] = time.monotonic()
            ctx.collect(DynamicInput(f"{self.model}_1", (1.0 + (i % 3), 1.0, 1.0, 1.0), occurred_on=i))

    def cancel(self):
        self._running = False


class IdleControl(SourceFunction):
    """One Add right away, then silence for ``idle_s`` (a control stream with sporadic messages)."""

    def __init__(self, path, idle_s):
        self.path = path
        self.idle_s = idle_s

    def run(self, ctx):
        ctx.collect(AddMessage(N1, 1, self.path, 0))
        time.sleep(self.idle_s)


def test_idle_control_source_does_not_stall_events(fixtures_dir):
    """10 Hz events + a control source idle for 2 s: every event is scored and emitted within
    max_batch_latency_ms + epsilon of its emission (round 2 measured 1.4 s late)."""
    from flink_jpmml_amd.api.pmml_model import PmmlModel

    PmmlModel.from_path(fixtures_dir["kmeans"])  # warm the parser (first-load imports)
    emitted = {}
    log = {}
    env = StreamExecutionEnvironment()
    events = env.add_source(PacedEvents(15, 0.1, log=log))
    control = env.add_source(IdleControl(fixtures_dir["kmeans"], 2.0))
    cfg = ScoringConfig(batch_size=64, max_batch_latency_ms=20.0)

    def sink(x):
        emitted[x[0]] = time.monotonic()

    events.with_support_stream(control).evaluate(
        lambda e, m: (e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)), config=cfg).add_sink(sink)
    t0 = time.monotonic()
    res = env.execute("live")
    assert res.input_mode == "live"
    assert sorted(emitted) == list(range(15))
    lat = {i: emitted[i] - log[i] for i in emitted}
    # events of the first ~0.1 s can race the Add (EmptyScore) but are never held back until the
    # idle control source yields (the round-2 bug: 1.4 s); the bound leaves room for a loaded host
    assert max(lat.values()) < 0.020 + 0.9, lat
    # the job ends when the idle control source finishes (2 s), not earlier
    assert time.monotonic() - t0 >= 1.9


def test_live_output_scores_match_after_add(fixtures_dir):
    out = []
    env = StreamExecutionEnvironment()
    events = env.add_source(PacedEvents(6, 0.05))
    control = env.add_source(IdleControl(fixtures_dir["kmeans"], 0.5))
    events.with_support_stream(control).evaluate(
        lambda e, m: (e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0))).add_sink(out.append)
    env.execute()
    # after the Add lands every event is scored; kmeans maps (1|2|3,1,1,1) to cluster 3.0
    assert [s for _, s in out][-3:] == [3.0, 3.0, 3.0]


# ------------------------------------------------------------------ socket source


class _LineServer:
    """A TCP server the test writes lines to, mid-run (nc -lk 9999 in the reference's README)."""

    def __init__(self):
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(1)
        self.port = self.srv.getsockname()[1]
        self.conn = None
        self._acc = threading.Thread(target=self._accept, daemon=True)
        self._acc.start()

    def _accept(self):
        self.conn, _ = self.srv.accept()

    def send(self, line):
        deadline = time.monotonic() + 10
        while self.conn is None and time.monotonic() < deadline:
            time.sleep(0.01)
        self.conn.sendall((line + "\n").encode())

    def close(self):
        if self.conn is not None:
            self.conn.close()
        self.srv.close()


def test_socket_text_stream_reads_lines_live():
    srv = _LineServer()
    got = []
    env = StreamExecutionEnvironment()
    env.socket_text_stream("127.0.0.1", srv.port).add_sink(lambda x: got.append((x, time.monotonic())))
    t = threading.Thread(target=env.execute, daemon=True)
    t.start()
    srv.send("first")
    time.sleep(0.3)
    assert [g for g, _ in got] == ["first"]  # delivered while the connection stays open
    srv.send("second")
    srv.send("third")
    time.sleep(0.2)
    srv.close()
    t.join(10)
    assert not t.is_alive()
    assert [g for g, _ in got] == ["first", "second", "third"]


def test_checkpoint_evaluate_example_streams_socket_and_output(fixtures_dir, tmp_path):
    """X4 end to end: the job scores while model paths are written to its socket mid-run, and its
    output file grows during the run (reference `E/CheckpointEvaluate.scala:56-98`)."""
    from flink_jpmml_amd.examples import jobs

    srv = _LineServer()
    out = tmp_path / "out.txt"
    args = jobs.build_parser().parse_args([
        "checkpoint", "--socket", f"127.0.0.1:{srv.port}", "--output", str(out), "--records", "40",
        "--rate", "20", "--intervalCheckpoint", "200", "--checkpoint-dir", str(tmp_path / "ck")])
    t = threading.Thread(target=jobs.checkpoint_evaluate, args=(args,), daemon=True)
    t.start()
    time.sleep(0.6)
    n0 = len(out.read_text().splitlines()) if out.exists() else 0
    assert n0 > 0  # events are scored (EmptyScore) before any model arrived
    srv.send(fixtures_dir["kmeans"])
    srv.send(fixtures_dir["kmeans"])
    time.sleep(0.8)
    n1 = len(out.read_text().splitlines())
    assert n1 > n0  # the file grows while the job runs
    srv.close()
    t.join(30)
    assert not t.is_alive()
    lines = out.read_text().splitlines()
    assert len(lines) == 40
    scored = [x.endswith("EmptyScore)") is False and ", Score(" in x for x in lines]
    # (event, EmptyScore) before the Add; (event, Score(..)) after it for the id(s) the paths got
    assert not scored[0] and sum(scored[n1:]) > 0
    assert CheckpointStorage(str(tmp_path / "ck")).latest() is not None  # time-based checkpoints ran


# ------------------------------------------------------------------ time-based checkpoints


def test_time_based_checkpoints_and_exact_restore(fixtures_dir, tmp_path):
    """Checkpoints every 50 ms on a live job; restoring from a mid-run manifest and replaying the
    rest yields exactly the uninterrupted output (offsets are the processed cut)."""
    k = fixtures_dir["kmeans"]
    ev = [DynamicInput(f"{N1}_1", (1.0 + (i % 5) / 2, 2.0, 3.0, 1.0), occurred_on=i) for i in range(60)]

    class Paced(SourceFunction):
        live = True

        def __init__(self, items, dt):
            self.items, self.dt = items, dt

        def _paced(self, items):
            # the control element (the model) is applied before the first event even on a loaded
            # machine: an event scored before it would be EmptyScore in one run and not the other
            time.sleep(0.3)
            for x in items:
                time.sleep(self.dt)
                yield x

        def iterate(self):
            return self._paced(self.items)

        def seek(self, off):
            return self._paced(self.items[off:])

    def job(out_dir, ck, restore=None, fail_after=None):
        env = StreamExecutionEnvironment()
        env.enable_checkpointing(interval_ms=50, directory=ck)
        if fail_after is not None:
            env.inject_failure(fail_after)
        events = env.add_source(Paced(ev, 0.005), uid="events")
        control = env.from_collection([AddMessage(N1, 1, k, 0)], uid="control")
        events.with_support_stream(control).evaluate(
            lambda e, m: [e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)], uid="scorer",
        ).add_sink(FileSink(out_dir))
        return env.execute("timed", restore=restore)

    ref = job(str(tmp_path / "ref"), str(tmp_path / "ref-ck"))
    assert ref.input_mode == "live" and len(ref.checkpoints) >= 2
    expected = FileSink.read(str(tmp_path / "ref"))
    assert len(expected) == 60
    with pytest.raises(Exception):
        job(str(tmp_path / "out"), str(tmp_path / "ck"), fail_after=45)
    latest = CheckpointStorage(str(tmp_path / "ck")).latest()
    doc = CheckpointStorage.read(latest)
    assert doc["trigger"] == "time" and 0 < doc["sources"]["events"]["offset"] < 60
    job(str(tmp_path / "out"), str(tmp_path / "ck"), restore=latest)
    got = FileSink.read(str(tmp_path / "out"))
    assert sorted(map(tuple, got)) == sorted(map(tuple, expected))


def test_time_based_checkpoints_with_manual_clock(fixtures_dir, tmp_path):
    """Deterministic input + virtual time: a checkpoint each time 1 s of job time has passed."""
    from flink_jpmml_amd.stream import ManualClock
    from flink_jpmml_amd.stream.clock import current_clock

    class Slow:
        def __iter__(self):
            for i in range(10):
                current_clock().sleep(0.25)
                yield DenseVector(1.0, 1.0, 1.0, float(i))

    env = StreamExecutionEnvironment(clock=ManualClock())
    env.enable_checkpointing(interval_ms=1000, directory=str(tmp_path))
    env.add_source(Slow()).quick_evaluate(__import__("flink_jpmml_amd").ModelReader(fixtures_dir["kmeans"])) \
        .add_sink(lambda x: None)
    res = env.execute()
    assert res.input_mode == "deterministic"
    assert len(res.checkpoints) == 2  # at t = 1.0 s and t = 2.0 s of 2.5 s


# ------------------------------------------------------------------ exact offsets


def test_timestamp_merge_checkpoint_does_not_skip_buffered_control(fixtures_dir, tmp_path):
    """Two timestamped sources, count checkpoints: the control element pre-read into the merge heap
    at the barrier (a Del) must be re-read after restore, not skipped."""
    k = fixtures_dir["kmeans"]
    events = [DynamicInput(f"{N1}_1", (1.0, 1.0, 1.0, 1.0), occurred_on=t) for t in range(0, 20, 2)]
    ctrl = [AddMessage(N1, 1, k, -1), DelMessage(N1, 1, 9)]

    def job(out_dir, ck, restore=None, fail_after=None):
        env = StreamExecutionEnvironment()
        env.enable_checkpointing(every_n_records=4, directory=ck)
        if fail_after is not None:
            env.inject_failure(fail_after)
        ev = env.from_collection(events, timestamp=lambda e: e.occurred_on, uid="events")
        cs = env.from_collection(ctrl, timestamp=lambda m: m.occurred_on, uid="control")
        ev.with_support_stream(cs).evaluate(
            lambda e, m: [e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)], uid="scorer",
        ).add_sink(FileSink(out_dir))
        return env.execute("ts", restore=restore)

    job(str(tmp_path / "ref"), str(tmp_path / "ref-ck"))
    expected = sorted(map(tuple, FileSink.read(str(tmp_path / "ref"))))
    assert [s for _, s in expected] == [3.0] * 5 + [-1.0] * 5  # Del at t=9 empties events from t=10
    with pytest.raises(Exception):
        job(str(tmp_path / "out"), str(tmp_path / "ck"), fail_after=9)
    ck = CheckpointStorage(str(tmp_path / "ck"))
    doc = CheckpointStorage.read(ck.latest())
    # barrier at event offset 4 (t=8): the Del (t=9) sat in the heap but was not processed
    assert doc["sources"]["control"]["offset"] == 1
    job(str(tmp_path / "out"), str(tmp_path / "ck"), restore=ck.latest())
    assert sorted(map(tuple, FileSink.read(str(tmp_path / "out")))) == expected


def test_file_sink_recover_commits_restored_pending_parts(tmp_path):
    """The process died after the manifest of checkpoint 2 was written but before commit(2):
    recover(2) publishes part 2 and drops part 3."""
    d = str(tmp_path / "sink")
    s = FileSink(d)
    s.open()
    for cid in (1, 2, 3):
        s.invoke([cid])
        s.pre_commit(cid)
    s.commit(1)
    s2 = FileSink(d)
    s2.open()
    s2.recover(2)
    assert FileSink.read(d) == [[1], [2]]
    assert not [f for f in os.listdir(d) if f.endswith(".pending")]


def test_records_in_counts_rows_of_batches():
    import numpy as np

    env = StreamExecutionEnvironment()
    env.from_batches(np.zeros((1000, 4)), batch_rows=300).add_sink(lambda x: None)
    res = env.execute()
    assert res.records_in == 1000 and res.elements_in == 4


def test_text_sink_streams_lines(tmp_path):
    path = tmp_path / "o.txt"
    seen = []

    class Src(SourceFunction):
        def run(self, ctx):
            for i in range(3):
                ctx.collect(i)
                time.sleep(0.15)
                seen.append(path.read_text().splitlines() if path.exists() else [])

    env = StreamExecutionEnvironment()
    env.add_source(Src()).write_as_text(str(path))
    env.execute()
    assert seen[0] == ["0"] and seen[1] == ["0", "1"]
    assert path.read_text().splitlines() == ["0", "1", "2"]


def test_manifest_is_json(tmp_path):
    env = StreamExecutionEnvironment()
    env.enable_checkpointing(every_n_records=2, directory=str(tmp_path))
    env.from_collection(list(range(5))).add_sink(lambda x: None)
    res = env.execute()
    with open(res.checkpoints[0]) as fh:
        doc = json.load(fh)
    assert doc["trigger"] == "count" and doc["checkpoint_id"] == 1


def test_gather_sink_pre_commit_retires_inflight_gathers():
    """the asynchronous device gather leaves collectives in flight after ``flush``; the
    checkpoint barrier (``pre_commit``) must retire them so no committed offset runs past rows the
    sink never delivered."""
    from flink_jpmml_amd.parallel.sinks import GatherSink

    sink = GatherSink(to="all")
    delivered = []
    for i in range(3):
        sink._inflight.append(([], [], lambda i=i: delivered.append(i)))
    sink.pre_commit(1)
    assert delivered == [0, 1, 2] and not sink._inflight
