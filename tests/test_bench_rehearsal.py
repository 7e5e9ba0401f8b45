"""The driver's N-rank ``bench.py`` launch, rehearsed on the CPU.

``python -m torch.distributed.run --nproc-per-node N ... bench.py --rehearse-cpu`` runs the exact
DSL job, GatherSink (lockstep all-gather, host path over gloo) and collective code of the timed
region with the host oracle scorer; every rank then checks every rank's gathered rows against
that rank's oracle scores. The committed 8-rank run is ``profiles/r4_rehearsal/``."""

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


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
