"""The driver's N-rank ``bench.py`` launch, rehearsed on the CPU.

``python -m torch.distributed.run --nproc-per-node N ... bench.py --rehearse-cpu`` runs the exact
DSL job, GatherSink (lockstep all-gather, host path over gloo) and collective code of the timed
region with the host oracle scorer; every rank then checks every rank's gathered rows against
that rank's oracle scores. The committed 8-rank run is ``profiles/r4_rehearsal/``.

Round 5: the check is per rank, over every gathered element, with the row
order taken from the source offsets — so it covers every bench mode: ``--models N`` (mixed-model
rows, each against its own model's oracle), ``--source binary`` (memory-mapped record files,
micro-batch elements) and ``--source text`` (CSV through the native parser), at world 8
(``profiles/r5_rehearsal/``)."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rehearse(tmp_path, world, *extra):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus",
           str(world), "--rehearse-cpu", "--rows", "512", "--passes", "2", "--steps", "1", "--warmup", "1",
           "--trees", "12", "--check-rows", "128", "--latency-iters", "2", "--ingest-threads", "1", *extra]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", [("--models", "16"), ("--source", "binary", "--micro-batch", "200"),
                                  ("--source", "text", "--micro-batch", "200")])
def test_bench_eight_rank_rehearsal_every_mode(tmp_path, mode):
    out = _rehearse(tmp_path, 8, *mode)
    assert out["n_gpus"] == 8 and out["rehearsal_cpu"]
    assert out["job"]["rehearsal_gather_check"] == [True] * 8
    assert out["job"]["rehearsal_rows_checked_per_rank"] == [512 * 2 * 2] * 8  # rows x passes x steps
    assert out["job"]["rehearsal_rows_gathered_per_rank"] == 8 * 512 * 2 * 2


def test_rehearsal_check_catches_misplaced_rows():
    """The per-rank check fails when two ranks' chunks are swapped inside a gathered element."""
    from types import SimpleNamespace

    import numpy as np

    sys.path.insert(0, ROOT)
    import bench

    args = SimpleNamespace(rows=64, features=4, source="synthetic", models=1, warmup=0, steps=1, passes=1)
    from flink_jpmml_amd.bench import synth

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_reh_model.pmml")
    with open(path, "w") as fh:
        fh.write(synth.gbdt_pmml(n_trees=5, depth=3, n_features=4, seed=3))
    try:
        parts = []
        for r in range(2):
            s, v = bench._rehearsal_reference(args, r, [path])
            parts.append((s.astype(np.float32), v, np.arange(64)))
        good = tuple(np.concatenate([p[i] for p in parts]) for i in range(3))
        swapped = tuple(np.concatenate([p[i] for p in parts[::-1]]) for i in range(3))
        for me in range(2):
            ctx = SimpleNamespace(world_size=2, rank=me)
            assert bench._rehearsal_check(args, SimpleNamespace(_parts=[good]), ctx, [path])[0]
            assert not bench._rehearsal_check(args, SimpleNamespace(_parts=[swapped]), ctx, [path])[0]
    finally:
        os.unlink(path)


def test_bench_spawns_its_own_ranks_without_a_launcher(tmp_path):
    """the driver's bare ``bench.py --gpus N`` (no torchrun, no WORLD_SIZE) must
    run N ranks — the parent spawns them and relays rank 0's JSON line."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR", "FJA_BENCH_CHILD"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--rehearse-cpu", "--rows", "512",
           "--passes", "2", "--steps", "1", "--warmup", "1", "--trees", "12", "--check-rows", "128",
           "--latency-iters", "2"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # exactly one JSON line: rank 0's
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["job"]["rehearsal_gather_check"] == [True] * 4


def test_bench_launcher_fails_when_a_rank_fails(tmp_path):
    """A rank that dies makes the launcher exit non-zero (the siblings are torn down)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR", "FJA_BENCH_CHILD"):
        env.pop(k, None)
    # --models with a file source is refused inside every rank (SystemExit) after the group formed
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-cpu", "--rows", "256",
           "--passes", "1", "--steps", "1", "--warmup", "1", "--trees", "4", "--check-rows", "0",
           "--models", "2", "--source", "binary"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert not any(ln.lstrip().startswith("{") for ln in r.stdout.splitlines())


def test_bench_two_rank_cpu_rehearsal(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--rehearse-cpu", "--rows", "1024", "--passes", "2", "--steps", "2", "--warmup", "1", "--trees", "20",
           "--check-rows", "256", "--latency-iters", "2"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and out["rehearsal_cpu"] and out["metric"].startswith("[CPU REHEARSAL")
    assert out["job"]["rehearsal_gather_check"] == [True, True]
    assert out["job"]["rehearsal_rows_gathered_per_rank"] == 2 * 1024 * 2 * 3  # ranks x rows x passes x steps
    assert out["check"]["valid_match"]
