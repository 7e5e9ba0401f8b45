"""Job launcher with a restart strategy — the MI355X form of Flink's fixed-delay restart.

The reference's fault-tolerance story (`flink-jpmml-examples/README.md:56-68`): kill a TaskManager
while ``CheckpointEvaluate`` runs, and Flink's restart strategy brings the job back from the last
completed checkpoint — the serving metadata is restored and models are re-read from their paths
(`S/api/functions/EvaluationCoFunction.scala:81-96`); no model has to be re-sent.

:class:`Supervisor` does that for a one-process-per-GPU job:

* it starts ``nproc`` ranks as **fresh child processes** (``RANK`` / ``LOCAL_RANK`` /
  ``WORLD_SIZE`` / ``MASTER_ADDR`` / ``MASTER_PORT`` in their environment, like ``torchrun``), each in
  its own session so it can be stopped as a whole process group;
* it never touches the GPU itself and never ``exec``s: a failed attempt's processes are killed and a
  new set of processes is spawned;
* when any rank exits non-zero (an injected kill, a watchdog abort after a peer stalled in a
  collective, a crash) the remaining ranks are stopped (SIGTERM, then SIGKILL after a grace period),
  and after ``restart_delay_s`` all ranks are relaunched with ``FJA_RESTORE`` set to
  :meth:`CheckpointStorage.latest` of the job's checkpoint directory (``FJA_CHECKPOINT_DIR``) —
  :meth:`StreamExecutionEnvironment.execute` restores from it when no explicit ``restore=`` is
  given — up to ``max_restarts`` times; ``FJA_ATTEMPT`` tells the job which attempt it is.

    python -m flink_jpmml_amd.launch --nproc 8 --max-restarts 3 --restart-delay 2 \\
        --checkpoint-dir /ckpt -- python my_job.py --output out/
"""

from __future__ import annotations

import argparse
import logging
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

logger = logging.getLogger(__name__)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@dataclass
class Attempt:
    index: int
    restore: Optional[str]
    exit_codes: List[Optional[int]] = field(default_factory=list)
    seconds: float = 0.0
    first_failure: Optional[int] = None  # exit code of the rank that failed first

    @property
    def ok(self) -> bool:
        return bool(self.exit_codes) and all(c == 0 for c in self.exit_codes)


class Supervisor:
    def __init__(self, cmd: Sequence[str], nproc: int, checkpoint_dir: Optional[str] = None, max_restarts: int = 3,
                 restart_delay_s: float = 1.0, grace_s: float = 5.0, env: Optional[Dict[str, str]] = None,
                 master_addr: str = "127.0.0.1", attempt_timeout_s: Optional[float] = None):
        self.cmd = list(cmd)
        self.nproc = int(nproc)
        self.checkpoint_dir = checkpoint_dir
        self.max_restarts = int(max_restarts)
        self.restart_delay_s = float(restart_delay_s)
        self.grace_s = float(grace_s)
        self.env = dict(env if env is not None else os.environ)
        self.master_addr = master_addr
        self.attempt_timeout_s = attempt_timeout_s
        self.attempts: List[Attempt] = []

    # ------------------------------------------------------------------ one attempt
    def _latest(self) -> Optional[str]:
        if not self.checkpoint_dir or not os.path.isdir(self.checkpoint_dir):
            return None
        from .stream.state import CheckpointStorage

        return CheckpointStorage(self.checkpoint_dir).latest()

    def _spawn(self, attempt: Attempt) -> List[subprocess.Popen]:
        port = _free_port()
        procs = []
        for r in range(self.nproc):
            env = dict(self.env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(self.nproc),
                       LOCAL_WORLD_SIZE=str(self.nproc), MASTER_ADDR=self.master_addr, MASTER_PORT=str(port),
                       FJA_ATTEMPT=str(attempt.index))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            if self.checkpoint_dir:
                env["FJA_CHECKPOINT_DIR"] = self.checkpoint_dir
            if attempt.restore:
                env["FJA_RESTORE"] = attempt.restore
            else:
                env.pop("FJA_RESTORE", None)
            procs.append(subprocess.Popen(self.cmd, env=env, start_new_session=True))
        return procs

    def _stop(self, procs: List[subprocess.Popen]) -> None:
        for sig, wait in ((signal.SIGTERM, self.grace_s), (signal.SIGKILL, 5.0)):
            alive = [p for p in procs if p.poll() is None]
            if not alive:
                return
            for p in alive:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass
            deadline = time.monotonic() + wait
            while time.monotonic() < deadline and any(p.poll() is None for p in alive):
                time.sleep(0.05)

    def _run_attempt(self, attempt: Attempt) -> None:
        t0 = time.monotonic()
        procs = self._spawn(attempt)
        failed = True  # stays set if the supervisor itself is interrupted: the ranks are stopped
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [c for c in codes if c not in (None, 0)]
                if bad:
                    attempt.first_failure = bad[0]
                    break
                if all(c == 0 for c in codes):
                    failed = False
                    break
                if self.attempt_timeout_s and time.monotonic() - t0 > self.attempt_timeout_s:
                    logger.error("attempt %d exceeded %.0f s", attempt.index, self.attempt_timeout_s)
                    break
                time.sleep(0.05)
        finally:
            if failed:
                self._stop(procs)
            else:
                for p in procs:
                    p.wait()
        attempt.exit_codes = [p.returncode for p in procs]
        attempt.seconds = time.monotonic() - t0

    # ------------------------------------------------------------------ restart strategy
    def run(self) -> int:
        """Run until an attempt succeeds (returns 0) or the restarts are exhausted (returns the
        failing attempt's first non-zero exit code)."""
        restore = os.environ.get("FJA_RESTORE") or None
        for i in range(self.max_restarts + 1):
            attempt = Attempt(i, restore)
            self.attempts.append(attempt)
            logger.info("attempt %d: %d rank(s)%s", i, self.nproc, f", restoring {restore}" if restore else "")
            self._run_attempt(attempt)
            if attempt.ok:
                return 0
            logger.error("attempt %d failed: exit codes %s", i, attempt.exit_codes)
            if i == self.max_restarts:
                break
            time.sleep(self.restart_delay_s)
            restore = self._latest() or restore
        code = self.attempts[-1].first_failure
        return int(code) if code is not None and code > 0 else 1


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        i = argv.index("--")
        own, cmd = argv[:i], argv[i + 1:]
    else:
        own, cmd = argv, []
    p = argparse.ArgumentParser(prog="python -m flink_jpmml_amd.launch")
    p.add_argument("--nproc", type=int, default=1, help="ranks (one per GPU)")
    p.add_argument("--max-restarts", type=int, default=3)
    p.add_argument("--restart-delay", type=float, default=1.0, help="seconds between attempts")
    p.add_argument("--grace", type=float, default=5.0, help="SIGTERM grace period before SIGKILL")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--attempt-timeout", type=float, default=None)
    a = p.parse_args(own)
    if not cmd:
        p.error("give the job command after --")
    logging.basicConfig(level=logging.INFO, format="[launch] %(message)s")

    def _terminate(signum, frame):  # SIGTERM to the supervisor: stop the ranks' process groups too
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, _terminate)
    sup = Supervisor(cmd, a.nproc, a.checkpoint_dir, a.max_restarts, a.restart_delay, a.grace,
                     attempt_timeout_s=a.attempt_timeout)
    return sup.run()


if __name__ == "__main__":
    sys.exit(main())
