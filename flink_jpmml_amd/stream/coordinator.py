"""Time-based checkpoint triggering across ranks (the JobManager's checkpoint coordinator).

The reference checkpoints on a wall-clock interval (`E/DynamicEvaluateKmeans.scala:48`,
`E/CheckpointEvaluate.scala:53`; ``--intervalCheckpoint`` is in ms, `E/util/DynamicParams.scala:38`).
Flink's JobManager decides when; every source task injects the barrier into its stream.

Here every rank runs one :class:`CheckpointCoordinator` thread on a dedicated gloo process group
(``"ckpt"``: no other thread uses it, so its collectives never interleave with the job thread's).
The threads meet in one small all-reduce per ``tick``:

* rank 0 contributes the id of the checkpoint to trigger (0 when the interval has not elapsed);
* every rank contributes 1 once its job thread has finished its input.

After the reduce all ranks know the same ``(trigger, done)``: a trigger becomes a barrier
:class:`~flink_jpmml_amd.stream.inputs.Marker` in every rank's input FIFO (each rank snapshots at
its own exact cut; the job threads then gather the state to rank 0 on the ``ctrl`` group, in
checkpoint-id order). When every rank is done a ``stop`` marker ends the job on every rank — a
rank that ran out of input keeps serving its peers' checkpoints until then, so the per-checkpoint
collectives always match.
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Optional

from .inputs import Marker

logger = logging.getLogger(__name__)


class CheckpointCoordinator:
    def __init__(self, ctx, interval_s: float, inject, first_cid: int = 1, tick_s: Optional[float] = None):
        self.ctx = ctx
        self.interval_s = float(interval_s)
        self.inject = inject  # callable(Marker), thread-safe (LiveInputs.inject)
        self.next_cid = int(first_cid)
        self.tick_s = float(tick_s if tick_s is not None else min(0.02, self.interval_s / 4))
        self.local_done = threading.Event()
        self._halt = threading.Event()
        self.rounds = 0
        self._t = threading.Thread(target=self._run, name=f"ckpt-coordinator-{ctx.rank}", daemon=True)

    def start(self) -> "CheckpointCoordinator":
        self._t.start()
        return self

    def _run(self) -> None:
        import torch
        import torch.distributed as dist

        group = self.ctx.group("ckpt")
        next_due = time.monotonic() + self.interval_s
        try:
            while not self._halt.is_set():
                time.sleep(self.tick_s)
                trig = 0
                if self.ctx.rank == 0 and time.monotonic() >= next_due:
                    trig = self.next_cid
                t = torch.tensor([trig, 1 if self.local_done.is_set() else 0], dtype=torch.int64)
                dist.all_reduce(t, group=group)
                self.rounds += 1
                trig, done = (int(x) for x in t.tolist())
                if done >= self.ctx.world_size:
                    self.inject(Marker("stop"))
                    return
                if trig:
                    self.next_cid = trig + 1
                    self.inject(Marker("barrier", trig))
                    if self.ctx.rank == 0:
                        next_due = time.monotonic() + self.interval_s
        except BaseException as e:  # noqa: BLE001 - a peer died: fail the job on the job thread
            from ..utils.faults import RankFailure

            if not self._halt.is_set():
                err = RankFailure(f"checkpoint coordinator: a peer rank is gone or stalled ({e})")
                err.__cause__ = e
                self.inject(Marker("error", exc=err))

    def finish_input(self) -> None:
        self.local_done.set()

    def stop(self) -> None:
        self._halt.set()
        if self._t.is_alive() and threading.current_thread() is not self._t:
            self._t.join(timeout=2 * self.tick_s + 5)


__all__ = ["CheckpointCoordinator"]
