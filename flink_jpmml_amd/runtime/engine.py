"""Pipelined micro-batch scoring engine (host records → GPU → host predictions).

The reference scores one record at a time on the JVM (`S/package.scala:76-79`). Here a stream of
records is scored in micro-batches through a three-stage pipeline on three HIP streams:

    H2D stream:   pinned host slice ──copy──▶ device input slot[i % depth]
    compute:      wait(H2D[i]) ▶ fused prepare + model kernel ▶ device score/valid (step buffer)
    D2H stream:   wait(compute[i]) ▶ score/valid slice ──copy──▶ pinned host output

A ring of ``depth`` device input slots lets batch i+1's copy overlap batch i's kernel and batch
i-1's copy-back. Nothing in :meth:`StreamingScorer.submit` blocks the host; :meth:`wait` is the
only synchronisation point. PCIe Gen5 (≈50+ GB/s per GPU) is the usual bound for wide fp32
records; the kernels themselves run far below it (see ``profiles/``).
"""

from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np


@dataclass
class StepHandle:
    n: int
    done: object  # torch.cuda.Event recorded on the D2H (or compute) stream
    score_dev: object = None
    valid_dev: object = None
    out_index: int = 0


class StreamingScorer:
    def __init__(self, plan, micro_batch: int = 131072, depth: int = 3, max_rows: Optional[int] = None,
                 out_buffers: int = 2, direct_host_output: bool = True, keep_device_output: bool = True,
                 h2d_streams: int = 1):
        import torch

        self.plan = plan
        self.device = plan.device
        self.F = plan.n_features
        self.B = int(micro_batch)
        self.depth = int(depth)
        # each micro-batch copy is split over `h2d_streams` streams: concurrent SDMA engines
        # (probe: 52.9 GB/s on one stream, 55.5 GB/s on four — profiles/r1_s3_probe_h2d*.json)
        self.h2ds = [torch.cuda.Stream(self.device) for _ in range(max(1, int(h2d_streams)))]
        self.h2d = self.h2ds[0]
        self.comp = torch.cuda.Stream(self.device)
        self.d2h = torch.cuda.Stream(self.device)
        self.x_slots = [torch.empty((self.B, self.F), dtype=torch.float32, device=self.device)
                        for _ in range(self.depth)]
        self.ev_h2d = [[torch.cuda.Event() for _ in self.h2ds] for _ in range(self.depth)]
        self.ev_comp = [torch.cuda.Event() for _ in range(self.depth)]
        self._used = [False] * self.depth
        self._slot = 0
        self.max_rows = max_rows or self.B
        # step output buffers, used round-robin: step k+1 never waits for step k's consumers
        self.n_out = int(out_buffers)
        self._outs = [self._alloc_out(self.max_rows) for _ in range(self.n_out)]
        self._out_free: List[Optional[object]] = [None] * self.n_out  # event: consumers of buffer done
        self._out_i = 0
        self.batch_times_ms: List[float] = []
        # zero-copy sink: the kernel epilogue writes scores straight into pinned host memory over
        # PCIe (no D2H copy commands: small D2H copies were measured to stall the H2D stream)
        self.direct = bool(direct_host_output) and getattr(plan, "supports_direct", False)
        self.keep_device = keep_device_output
        self._dev_ptr_cache = {}

    def _host_dev_ptr(self, t):
        from ..ops._lib import host_device_ptr

        key = (t.data_ptr(), t.numel())
        if key not in self._dev_ptr_cache:
            self._dev_ptr_cache[key] = host_device_ptr(t)
        return self._dev_ptr_cache[key]

    def _alloc_out(self, n: int):
        import torch

        return (torch.empty(n, dtype=torch.float32, device=self.device),
                torch.empty(n, dtype=torch.uint8, device=self.device))

    @property
    def score_dev(self):
        return self._outs[(self._out_i - 1) % self.n_out][0]

    @property
    def valid_dev(self):
        return self._outs[(self._out_i - 1) % self.n_out][1]

    def ensure_capacity(self, n: int) -> None:
        if n > self.max_rows:
            self.max_rows = n
            self._outs = [self._alloc_out(n) for _ in range(self.n_out)]
            self._out_free = [None] * self.n_out

    def submit(self, X_host, score_host=None, valid_host=None, offset: int = 0) -> StepHandle:
        """Enqueue scoring of a pinned host matrix ``X_host`` ([n, F] float32 tensor). Scores land in
        this step's device output buffer (``handle.score_dev``) and, if given, in the pinned host
        outputs. Returns immediately."""
        import torch

        n = int(X_host.shape[0])
        self.ensure_capacity(offset + n)
        oi = self._out_i
        self._out_i = (oi + 1) % self.n_out
        score_dev, valid_dev = self._outs[oi]
        if self._out_free[oi] is not None:
            self.comp.wait_event(self._out_free[oi])  # WAR: the step that last used this buffer
        hs = hv = None
        if self.direct and score_host is not None and valid_host is not None:
            hs, hv = self._host_dev_ptr(score_host), self._host_dev_ptr(valid_host)
            if hs is None or hv is None:
                hs = hv = None
        for s in range(0, n, self.B):
            e = min(n, s + self.B)
            m = e - s
            slot = self._slot
            self._slot = (slot + 1) % self.depth
            xs = self.x_slots[slot][:m]
            part = -(-m // len(self.h2ds))
            for j, st in enumerate(self.h2ds):
                with torch.cuda.stream(st):
                    if self._used[slot]:
                        st.wait_event(self.ev_comp[slot])  # kernel finished reading this slot
                    a, b = j * part, min(m, (j + 1) * part)
                    if a < b:
                        xs[a:b].copy_(X_host[s + a:s + b], non_blocking=True)
                    self.ev_h2d[slot][j].record(st)
            for ev in self.ev_h2d[slot]:
                self.comp.wait_event(ev)
            if hs is not None:
                kw = {}
                if self.keep_device:
                    kw = dict(score2=score_dev[offset + s: offset + e], valid2=valid_dev[offset + s: offset + e])
                self.plan.launch(xs, hs + 4 * s, hv + s, stream=self.comp, **kw)
            else:
                self.plan.launch(xs, score_dev[offset + s: offset + e], valid_dev[offset + s: offset + e],
                                 stream=self.comp)
            self.ev_comp[slot].record(self.comp)
            self._used[slot] = True
            if score_host is not None and hs is None:
                with torch.cuda.stream(self.d2h):
                    self.d2h.wait_event(self.ev_comp[slot])
                    score_host[s:e].copy_(score_dev[offset + s: offset + e], non_blocking=True)
                    if valid_host is not None:
                        valid_host[s:e].copy_(valid_dev[offset + s: offset + e], non_blocking=True)
        done = torch.cuda.Event()
        if score_host is not None and hs is None:
            done.record(self.d2h)
        else:
            done.record(self.comp)
        self._out_free[oi] = done
        h = StepHandle(n, done)
        h.score_dev = score_dev[offset: offset + n]
        h.valid_dev = valid_dev[offset: offset + n]
        h.out_index = oi
        return h

    def mark_consumed(self, handle: StepHandle, stream) -> None:
        """Declare that ``stream`` also reads this step's device outputs (e.g. an all-gather): the
        step that next reuses the buffer waits for it."""
        import torch

        ev = torch.cuda.Event()
        ev.record(stream)
        prev = self._out_free[handle.out_index]
        if prev is not None:
            stream.wait_event(prev)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._out_free[handle.out_index] = ev

    def join(self, stream=None) -> None:
        """Make ``stream`` (default: current) wait for all work submitted so far (no host sync)."""
        import torch

        s = stream or torch.cuda.current_stream(self.device)
        for st in (*self.h2ds, self.comp, self.d2h):
            ev = torch.cuda.Event()
            ev.record(st)
            s.wait_event(ev)

    @staticmethod
    def wait(handle: StepHandle) -> None:
        handle.done.synchronize()

    def score_numpy(self, X: np.ndarray) -> tuple:
        """Blocking convenience: score a host numpy matrix, return numpy ``(score, valid)``."""
        import torch

        Xp = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).pin_memory()
        sh = torch.empty(X.shape[0], dtype=torch.float32).pin_memory()
        vh = torch.empty(X.shape[0], dtype=torch.uint8).pin_memory()
        t0 = time.perf_counter()
        h = self.submit(Xp, sh, vh)
        self.wait(h)
        self.batch_times_ms.append((time.perf_counter() - t0) * 1e3)
        return sh.numpy().copy(), vh.numpy().astype(bool)
