"""The Flink-shaped DSL under data parallelism: one process per rank (gloo on CPU here; the same
code runs RCCL on GPUs under torchrun). Every rank builds the same job; operators run as one
subtask per rank; event streams are sharded, control streams replicated, models parsed once on
rank 0 and replicated, outputs all-gathered; checkpoints are aligned across ranks and a killed
rank is recovered from the manifest with exactly-once output (SURVEY §2.6 F1–F5, §5.3, §5.4)."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N1 = "a1b2c3d4-0000-4000-8000-000000000001"
N2 = "a1b2c3d4-0000-4000-8000-000000000002"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(world, fn, args, extra_env=None, timeout=180):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, extra_env or {})) for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    import time as _time

    results = {}
    deadline = _time.monotonic() + timeout
    try:
        while len(results) < world and _time.monotonic() < deadline:
            try:
                r, res = q.get(timeout=1.0)
                results[r] = res
            except _queue.Empty:
                if not any(p.is_alive() for p in procs):  # a killed rank never reports
                    break
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return results, [p.exitcode for p in procs]


def _entry(rank, world, port, fn, args, q, extra_env):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FJA_DIST_TIMEOUT_S="30", **extra_env)
    try:
        res = fn(*args)
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, ("error", type(e).__name__, str(e)[:300], type(e.__cause__).__name__ if e.__cause__ else None)))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001
                pass


# ------------------------------------------------------------------ jobs (run on every rank)


def _dynamic_seq(kmeans, notarget):
    from flink_jpmml_amd import AddMessage, DelMessage
    from tests.test_stream import DynamicInput

    seq, k = [], 0

    def ev(name, vals=(1.0, 1.0, 1.0, 1.0)):
        nonlocal k
        k += 1
        return ("L", DynamicInput(f"{name}_1", vals, occurred_on=k))

    seq += [ev(N1)]
    seq += [("R", AddMessage(N1, 1, kmeans, 0)), ("R", AddMessage(N2, 1, notarget, 0))]
    seq += [ev(N1, (1.0 + i / 7, 2.0, 3.0, 4.0 - i / 9)) for i in range(9)] + [ev(N2) for _ in range(3)]
    seq += [("R", DelMessage(N1, 1, 0))] + [ev(N1) for _ in range(3)]
    seq += [("R", AddMessage(N1, 2, kmeans, 0))] + [ev(N1.replace("1", "1"), (6.0, 3.0, 5.0, 2.0)) for _ in range(2)]
    return seq


def job_dynamic(kmeans, notarget, batch):
    from flink_jpmml_amd.stream import StreamExecutionEnvironment

    env = StreamExecutionEnvironment.get_execution_environment()
    assert env.is_distributed and env.parallelism == int(os.environ["WORLD_SIZE"])
    events, control = env.from_either(_dynamic_seq(kmeans, notarget))
    out = events.with_support_stream(control).evaluate(
        lambda e, m: (e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)), batch_size=batch).collect()
    return sorted(out)


def job_columnar(kmeans, n, batch_rows):
    import numpy as np

    from flink_jpmml_amd import ModelReader
    from flink_jpmml_amd.stream import StreamExecutionEnvironment
    from flink_jpmml_amd.utils.metrics import METRICS

    env = StreamExecutionEnvironment.get_execution_environment()
    X = np.random.default_rng(7).uniform(0.2, 7.0, size=(n, 4))
    out = env.from_batches(X, batch_rows=batch_rows).quick_evaluate(ModelReader(kmeans)).collect()
    offs = [b.offset for _, b in out]
    scores = np.concatenate([p.values(-1.0) for p, _ in out])
    order = np.argsort(np.concatenate([b.offset + np.arange(len(b)) for _, b in out]))
    return offs, scores[order].tolist(), METRICS.counters.get("model.loads_replicated", 0)


def job_exactly_once(kmeans, out_dir, ck_dir, restore):
    from flink_jpmml_amd.stream import FileSink, StreamExecutionEnvironment
    from tests.test_stream import DynamicInput

    from flink_jpmml_amd import AddMessage

    seq = [("R", AddMessage(N1, 1, kmeans, 0))] + \
          [("L", DynamicInput(f"{N1}_1", (1.0 + i / 10, 2.0, 3.0, 1.0), occurred_on=i)) for i in range(40)]
    env = StreamExecutionEnvironment.get_execution_environment()
    env.enable_checkpointing(every_n_records=8, directory=ck_dir)
    events, control = env.from_either(seq)
    events.with_support_stream(control).evaluate(
        lambda e, m: [e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)], uid="scorer"
    ).add_sink(FileSink(out_dir))
    env.execute("dist-exactly-once", restore=restore)
    return "done"


def job_midstream_adds_with_gather(kmeans, n_batches, rows):
    """Add messages arrive mid-stream while the library GatherSink all-gathers scored batches; every
    object collective of the loader thread is recorded with the process group it used."""
    import threading

    import numpy as np

    from flink_jpmml_amd import AddMessage
    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.parallel import dist as D
    from flink_jpmml_amd.parallel.sinks import GatherSink
    from flink_jpmml_amd.stream import StreamExecutionEnvironment

    calls = []
    orig = D.broadcast_object

    def spy(obj, ctx, src=0, group=None):
        name = next((k for k, g in ctx.groups.items() if g is group), None)
        calls.append((threading.current_thread().name, name))
        return orig(obj, ctx, src, group)

    D.broadcast_object = spy
    N3 = "a1b2c3d4-0000-4000-8000-000000000003"
    rng = np.random.default_rng(3)
    seq = [("R", AddMessage(N1, 1, kmeans, 0))]
    for i in range(n_batches):
        X = rng.uniform(0.2, 7.0, size=(rows, 4))
        ids = [N1, N2, N3][i % 3] if i >= 6 else N1
        seq.append(("L", RecordBatch(X, model_id=f"{ids}_1", offset=i * rows)))
        if i == 3:
            seq.append(("R", AddMessage(N2, 1, kmeans, 0)))  # mid-stream, while gathers are in flight
        if i == 5:
            seq.append(("R", AddMessage(N3, 1, kmeans, 0)))
    env = StreamExecutionEnvironment.get_execution_environment()
    events, control = env.from_either(seq)
    sink = GatherSink(to="all")
    events.with_support_stream(control).quick_evaluate().add_sink(sink)
    env.execute("midstream-adds")
    sink.finish()
    loader = [(t, g) for t, g in calls if t.startswith("model-loader")]
    order = np.argsort(sink.offsets)
    return loader, sink.scores[order].tolist(), sink.valid[order].tolist(), sink.offsets[order].tolist()


# ------------------------------------------------------------------ tests


def _single_process_dynamic(kmeans, notarget):
    from flink_jpmml_amd.stream import StreamExecutionEnvironment

    env = StreamExecutionEnvironment()
    events, control = env.from_either(_dynamic_seq(kmeans, notarget))
    return sorted(events.with_support_stream(control).evaluate(
        lambda e, m: (e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0))).collect())


@pytest.mark.parametrize("world,batch", [(2, None), (4, None), (2, 3), (4, 2)])
def test_dynamic_job_dp(fixtures_dir, world, batch):
    """The 15-scenario dynamic-serving contract, sharded over `world` ranks: identical outputs."""
    ref = _single_process_dynamic(fixtures_dir["kmeans"], fixtures_dir["kmeans_nooutput_notarget"])
    res, codes = _spawn(world, job_dynamic, (fixtures_dir["kmeans"], fixtures_dir["kmeans_nooutput_notarget"], batch))
    assert codes == [0] * world, res
    for r in range(world):
        assert res[r] == ref, res[r]
    assert sum(1 for _, s in ref if s == -1.0) >= 7 and sum(1 for _, s in ref if s != -1.0) >= 9


def test_columnar_job_dp_shards_and_gathers(fixtures_dir):
    from flink_jpmml_amd.api.pmml_model import PmmlModel

    n, world = 1000, 2
    res, codes = _spawn(world, job_columnar, (fixtures_dir["kmeans"], n, 100))
    assert codes == [0] * world, res
    X = np.random.default_rng(7).uniform(0.2, 7.0, size=(n, 4))
    ref = PmmlModel.from_path(fixtures_dir["kmeans"]).predict(X).values(-1.0).tolist()
    for r in range(world):
        offs, scores, replicated = res[r]
        assert scores == ref
        assert offs == [0, 200, 400, 600, 800, 100, 300, 500, 700, 900]  # rank 0's shard, then rank 1's
        assert replicated == 1  # parsed once on rank 0, replicated (one collective load per rank)


def test_killed_rank_recovers_exactly_once(fixtures_dir, tmp_path):
    """kill_rank=1@9: rank 1 dies mid-stream; rank 0's next checkpoint collective raises
    RankFailure; restarting both ranks from the last aligned manifest yields exactly the
    uninterrupted run's committed output (no duplicates, no gaps)."""
    from flink_jpmml_amd.stream import FileSink
    from flink_jpmml_amd.stream.state import CheckpointStorage
    from flink_jpmml_amd.utils.faults import EXIT_KILLED_RANK

    k = fixtures_dir["kmeans"]
    ref_dir, ref_ck = str(tmp_path / "ref"), str(tmp_path / "ref-ck")
    res, codes = _spawn(2, job_exactly_once, (k, ref_dir, ref_ck, None))
    assert codes == [0, 0] and res[0] == "done", res
    expected = sorted(map(tuple, FileSink.read(ref_dir)))
    assert len(expected) == 40

    out_dir, ck = str(tmp_path / "out"), str(tmp_path / "ck")
    res, codes = _spawn(2, job_exactly_once, (k, out_dir, ck, None), extra_env={"FJA_FAULTS": "kill_rank=1@9"})
    assert codes[1] == EXIT_KILLED_RANK
    assert res[0][0] == "error" and res[0][1] == "JobExecutionException" and res[0][3] == "RankFailure", res
    latest = CheckpointStorage(ck).latest()
    assert latest is not None
    doc = CheckpointStorage.read(latest)
    assert doc["world_size"] == 2 and len(doc["operators"]["scorer"]["metadata-snapshot"]["subtasks"]) == 2
    partial = FileSink.read(out_dir)
    assert 0 < len(partial) < 40
    res, codes = _spawn(2, job_exactly_once, (k, out_dir, ck, latest))
    assert codes == [0, 0], res
    assert sorted(map(tuple, FileSink.read(out_dir))) == expected


# ------------------------------------------------------------------ live input + time-based checkpoints


class PacedShardSource:
    """A live (sleeping) replayable source, read on a reader thread; sharded by global offset."""

    live = True

    def __init__(self, items, dt):
        self.items = items
        self.dt = dt

    def iterate(self):
        import time

        for x in self.items:
            time.sleep(self.dt)
            yield x

    def seek(self, off):
        return iter(self.items[off:])


def job_timed_exactly_once(kmeans, out_dir, ck_dir, restore):
    from flink_jpmml_amd import AddMessage
    from flink_jpmml_amd.stream import FileSink, StreamExecutionEnvironment
    from tests.test_stream import DynamicInput

    ev = [DynamicInput(f"{N1}_1", (1.0 + (i % 7) / 3, 2.0, 3.0, 1.0), occurred_on=i) for i in range(60)]
    env = StreamExecutionEnvironment.get_execution_environment()
    env.enable_checkpointing(interval_ms=40, directory=ck_dir)
    events = env.add_source(PacedShardSource(ev, 0.008), uid="events")  # kill at 20 ≈ 160 ms: several 40 ms checkpoints even on a loaded host
    control = env.from_collection([AddMessage(N1, 1, kmeans, 0)], uid="control")
    events.with_support_stream(control).evaluate(
        lambda e, m: [e.occurred_on, m.predict(e.to_vector()).value.get_or_else(-1.0)], uid="scorer"
    ).add_sink(FileSink(out_dir))
    res = env.execute("dist-timed", restore=restore)
    return res.input_mode, len(res.checkpoints)


def test_time_based_checkpoints_across_ranks_recover_exactly_once(fixtures_dir, tmp_path):
    """Rank 0 triggers checkpoints every 40 ms (coordinator thread on its own gloo group); every
    rank snapshots its own exact cut. Killing rank 1 mid-stream and restoring both ranks from the
    last manifest gives exactly the uninterrupted run's output."""
    from flink_jpmml_amd.stream import FileSink
    from flink_jpmml_amd.stream.state import CheckpointStorage
    from flink_jpmml_amd.utils.faults import EXIT_KILLED_RANK

    k = fixtures_dir["kmeans"]
    ref_dir, ref_ck = str(tmp_path / "ref"), str(tmp_path / "ref-ck")
    res, codes = _spawn(2, job_timed_exactly_once, (k, ref_dir, ref_ck, None))
    assert codes == [0, 0], res
    assert res[0][0] == "live" and res[0][1] >= 1 and res[0][1] == res[1][1], res
    expected = sorted(map(tuple, FileSink.read(ref_dir)))
    assert len(expected) == 60 and all(s > 0 for _, s in expected[5:])

    out_dir, ck = str(tmp_path / "out"), str(tmp_path / "ck")
    res, codes = _spawn(2, job_timed_exactly_once, (k, out_dir, ck, None), extra_env={"FJA_FAULTS": "kill_rank=1@20"})
    assert codes[1] == EXIT_KILLED_RANK
    assert res[0][0] == "error" and res[0][1] == "JobExecutionException", res
    latest = CheckpointStorage(ck).latest()
    assert latest is not None
    doc = CheckpointStorage.read(latest)
    assert doc["trigger"] == "time" and len(doc["sources"]["events"]["ranks"]) == 2
    res, codes = _spawn(2, job_timed_exactly_once, (k, out_dir, ck, latest))
    assert codes == [0, 0], res
    got = sorted(map(tuple, FileSink.read(out_dir)))
    assert [i for i, _ in got] == [i for i, _ in expected]  # every event exactly once
    # identical scores, except that the first events of a run race the control stream's model
    # (EmptyScore -> -1 until the model is loaded, in the reference run or in the killed run's
    # committed prefix alike)
    assert all(a == b or -1.0 in (a, b) for (_, a), (_, b) in zip(got, expected)), (got, expected)
    assert got[10:] == expected[10:]


# ------------------------------------------------------------------ world 8


def test_dynamic_job_world8(fixtures_dir):
    """The 15-scenario dynamic-serving contract at world size 8 (gloo): identical outputs."""
    ref = _single_process_dynamic(fixtures_dir["kmeans"], fixtures_dir["kmeans_nooutput_notarget"])
    res, codes = _spawn(8, job_dynamic, (fixtures_dir["kmeans"], fixtures_dir["kmeans_nooutput_notarget"], 2),
                        timeout=300)
    assert codes == [0] * 8, res
    for r in range(8):
        assert res[r] == ref, res[r]


def job_columnar_gather(kmeans, n, batch_rows):
    import numpy as np

    from flink_jpmml_amd import ModelReader
    from flink_jpmml_amd.parallel.sinks import GatherSink
    from flink_jpmml_amd.stream import StreamExecutionEnvironment
    from flink_jpmml_amd.utils.metrics import METRICS

    env = StreamExecutionEnvironment.get_execution_environment()
    X = np.random.default_rng(7).uniform(0.2, 7.0, size=(n, 4))
    sink = GatherSink(to="all")
    env.from_batches(X, batch_rows=batch_rows).quick_evaluate(ModelReader(kmeans)).add_sink(sink)
    env.execute("gather")
    order = np.argsort(sink.offsets)
    return (sink.scores[order].tolist(), sink.valid[order].tolist(), METRICS.counters.get("source.foreign_elements", 0),
            len(sink.offsets))


@pytest.mark.parametrize("world", [2, 8])
def test_columnar_shard_and_library_gather_sink(fixtures_dir, world):
    """Rank-local shards (no rank materialises another's batches) + the library GatherSink: every
    rank ends with every row's score, in source order."""
    from flink_jpmml_amd.api.pmml_model import PmmlModel

    n = 1000
    res, codes = _spawn(world, job_columnar_gather, (fixtures_dir["kmeans"], n, 50), timeout=300)
    assert codes == [0] * world, res
    X = np.random.default_rng(7).uniform(0.2, 7.0, size=(n, 4))
    pb = PmmlModel.from_path(fixtures_dir["kmeans"]).predict(X)
    for r in range(world):
        scores, valid, foreign, rows = res[r]
        assert rows == n and foreign == 0
        assert scores == pb.scores.tolist() and valid == pb.valid.tolist()


def job_text_split(kmeans, path):
    from flink_jpmml_amd import ModelReader
    from flink_jpmml_amd.stream import StreamExecutionEnvironment
    from flink_jpmml_amd.utils.metrics import METRICS

    env = StreamExecutionEnvironment.get_execution_environment()
    out = env.read_text_batches(path, ModelReader(kmeans), batch_rows=64).quick_evaluate(
        ModelReader(kmeans)).collect()
    rows = sum(len(b) for _, b in out)
    return METRICS.counters.get("ingest.bytes_parsed", 0), rows


def test_text_source_splits_bytes_across_ranks(fixtures_dir, tmp_path):
    """4 ranks: every input byte is parsed by exactly one rank (counter), every row scored once."""
    from flink_jpmml_amd import native

    native.load()  # builds the g++ ingest if needed
    rng = np.random.default_rng(3)
    path = tmp_path / "in.csv"
    header = "sepal_length,sepal_width,petal_length,petal_width\n"
    lines = [",".join(f"{v:.3f}" for v in row) + "\n" for row in rng.uniform(0.2, 7.0, size=(997, 4))]
    path.write_text(header + "".join(lines))
    data_bytes = os.path.getsize(path) - len(header)
    res, codes = _spawn(4, job_text_split, (fixtures_dir["kmeans"], str(path)))
    assert codes == [0] * 4, res
    per_rank = [res[r][0] for r in range(4)]
    assert all(b > 0 for b in per_rank) and sum(per_rank) == data_bytes
    assert all(res[r][1] == 997 for r in range(4))  # collect() all-gathers every rank's rows


# ------------------------------------------------------------------ restart strategy

SUPERVISED_JOB = r"""
import os, sys
sys.path.insert(0, os.environ["FJA_ROOT"])
from tests.test_dist_dsl import job_exactly_once
kmeans, out_dir = sys.argv[1], sys.argv[2]
job_exactly_once(kmeans, out_dir, os.environ["FJA_CHECKPOINT_DIR"], None)
"""


def test_supervisor_restarts_killed_job_exactly_once(fixtures_dir, tmp_path):
    """kill_rank=1@9 on the first attempt: the supervisor sees the dead rank, stops the survivor,
    relaunches both ranks as fresh processes restoring CheckpointStorage.latest() on their own —
    the committed output equals the uninterrupted run's (no manual restore=)."""
    import sys

    from flink_jpmml_amd.launch import Supervisor
    from flink_jpmml_amd.stream import FileSink
    from flink_jpmml_amd.utils.faults import EXIT_KILLED_RANK

    k = fixtures_dir["kmeans"]
    ref_dir, ref_ck = str(tmp_path / "ref"), str(tmp_path / "ref-ck")
    res, codes = _spawn(2, job_exactly_once, (k, ref_dir, ref_ck, None))
    assert codes == [0, 0], res
    expected = sorted(map(tuple, FileSink.read(ref_dir)))

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out_dir, ck = str(tmp_path / "out"), str(tmp_path / "ck")
    env = dict(os.environ, FJA_ROOT=root, FJA_FAULTS="kill_rank=1@9", FJA_FAULT_ATTEMPTS="1",
               FJA_DIST_TIMEOUT_S="20")
    env.pop("FJA_RESTORE", None)
    sup = Supervisor([sys.executable, "-c", SUPERVISED_JOB, k, out_dir], nproc=2, checkpoint_dir=ck,
                     max_restarts=2, restart_delay_s=0.2, grace_s=2.0, env=env, attempt_timeout_s=150)
    assert sup.run() == 0
    assert len(sup.attempts) == 2
    assert EXIT_KILLED_RANK in sup.attempts[0].exit_codes
    assert sup.attempts[1].restore is not None and sup.attempts[1].ok
    assert sorted(map(tuple, FileSink.read(out_dir))) == expected


def test_supervisor_gives_up_after_max_restarts(tmp_path):
    import sys

    from flink_jpmml_amd.launch import Supervisor

    sup = Supervisor([sys.executable, "-c", "import sys; sys.exit(3)"], nproc=2, checkpoint_dir=str(tmp_path),
                     max_restarts=1, restart_delay_s=0.0, grace_s=0.5)
    assert sup.run() == 3 and len(sup.attempts) == 2


def test_supervisor_sigterm_stops_its_ranks(tmp_path):
    """SIGTERM to the launcher must not orphan the ranks (each runs in its own session)."""
    import os
    import signal
    import subprocess
    import sys
    import time

    pidfile = tmp_path / "pids"
    child = (f"import os, time; open({str(pidfile)!r} + os.environ['RANK'], 'w').write(str(os.getpid())); "
             "time.sleep(120)")
    sup = subprocess.Popen([sys.executable, "-m", "flink_jpmml_amd.launch", "--nproc", "2", "--grace", "0.5", "--",
                            sys.executable, "-c", child])
    try:
        deadline = time.monotonic() + 60
        while time.monotonic() < deadline and not all((tmp_path / f"pids{r}").exists() and (tmp_path / f"pids{r}").stat().st_size
                                                for r in range(2)):
            time.sleep(0.05)
        pids = [int((tmp_path / f"pids{r}").read_text()) for r in range(2)]
        sup.send_signal(signal.SIGTERM)
        assert sup.wait(timeout=30) != 0
        deadline = time.monotonic() + 10
        alive = pids
        while time.monotonic() < deadline and alive:
            alive = []
            for p in pids:
                try:
                    os.kill(p, 0)
                    alive.append(p)
                except ProcessLookupError:
                    pass
            time.sleep(0.05)
        assert not alive, f"ranks left running: {alive}"
    finally:
        if sup.poll() is None:
            sup.kill()


def test_replicated_loads_handshake_on_gloo_while_gathers_run(fixtures_dir):
    """with Add messages arriving mid-stream while GatherSink all-gathers run
    on the job thread, the loader thread's object handshake (header / errors / plan metadata) uses
    its own gloo group (``model_ctrl``) -- never the data-backend ``model`` group, which is RCCL on
    GPUs -- and every rank gathers the same, correct scores."""
    from flink_jpmml_amd.api.pmml_model import PmmlModel

    world, n_batches, rows = 4, 12, 50
    res, codes = _spawn(world, job_midstream_adds_with_gather, (fixtures_dir["kmeans"], n_batches, rows),
                        timeout=300)
    assert codes == [0] * world, res
    rng = np.random.default_rng(3)
    X = np.concatenate([rng.uniform(0.2, 7.0, size=(rows, 4)) for _ in range(n_batches)])
    ref = PmmlModel.from_path(fixtures_dir["kmeans"]).predict(X).values(-1.0)
    for r in range(world):
        loader, scores, valid, offs = res[r]
        assert len(loader) == 3, loader  # one handshake per Add, on the loader thread
        assert {g for _, g in loader} == {"model_ctrl"}, loader
        assert offs == list(range(n_batches * rows))
        assert all(valid)
        np.testing.assert_allclose(scores, ref, rtol=0, atol=1e-9)
