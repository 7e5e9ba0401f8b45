"""Library sinks for data-parallel scoring jobs (SURVEY §2.6 **F5**).

In the reference every parallel subtask writes its own output (`writeAsText`,
`E/EvaluateKmeans.scala:53`; the test sink, `T/utils/FlinkTestKits.scala:58-62`). On an MI355X node
the scored shards of all GPUs are combined with one collective instead:

:class:`GatherSink` receives the operators' columnar results — ``(PredictionBatch, RecordBatch)``
from ``quick_evaluate`` or a bare ``PredictionBatch`` — and gathers every rank's scores, validity
masks and source row offsets, to every rank (``to="all"``) or to rank 0 (``to=0``):

* **device path** (RCCL): when the batches carry device mirrors (``ScoringConfig(device_mirror=True)``
  keeps them) the scores never leave HBM; the gather runs ``all_gather_into_tensor`` over xGMI on a
  dedicated HIP stream that waits on the scoring kernel's completion event (no host sync), so it
  overlaps the next batch's H2D and kernel;
* **host path** (gloo, or models scored on the host): the pinned host arrays are gathered on the
  job thread's ``ctrl`` group.

Two cadences:

* ``lockstep=True`` — one gather per element. Every rank must produce the same number of elements
  with the same row count (synthetic per-rank streams such as ``bench.py``); sizes are checked once.
* default — elements are buffered and gathered at every checkpoint barrier (``pre_commit``) and at
  end of input, the points where all ranks meet anyway; variable lengths per rank.

``keep=True`` accumulates the gathered rows on the host (``scores`` / ``valid`` / ``offsets``,
rank-major order; sort by ``offsets`` for source order); ``on_gathered(scores, valid, offsets)`` is
called per gather round instead/as well.
"""

from __future__ import annotations

import logging
from typing import Any, Callable, List, Optional, Tuple

import numpy as np

from ..api.batch import PredictionBatch, RecordBatch
from ..stream.functions import SinkFunction
from ..utils.metrics import METRICS

logger = logging.getLogger(__name__)


def _split(value: Any) -> Tuple[PredictionBatch, Optional[RecordBatch]]:
    if isinstance(value, PredictionBatch):
        return value, None
    if isinstance(value, (tuple, list)) and value and isinstance(value[0], PredictionBatch):
        batch = value[1] if len(value) > 1 and isinstance(value[1], RecordBatch) else None
        return value[0], batch
    raise TypeError(f"GatherSink expects PredictionBatch or (PredictionBatch, RecordBatch) elements, got "
                    f"{type(value).__name__}")


def _row_offsets(pb: PredictionBatch, batch: Optional[RecordBatch]) -> np.ndarray:
    n = len(pb)
    if batch is None:
        return np.full(n, -1, dtype=np.int64)
    if batch.row_index is not None:
        return batch.offset + np.asarray(batch.row_index, dtype=np.int64)
    return batch.offset + np.arange(n, dtype=np.int64)


def gather_varlen(t, ctx, group=None, dst: Optional[int] = None):
    """Gather 1-D/2-D tensor shards of different lengths along dim 0, in rank order: to every rank
    (``dst=None``, ``all_gather_into_tensor``) or to ``dst`` (others get ``None``). Two collectives:
    the lengths, then the padded payload."""
    import torch
    import torch.distributed as dist

    if not ctx.is_distributed:
        return t
    dev = t.device
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(ctx.world_size)]
    dist.all_gather(sizes, n, group=group)
    sz = [int(s.item()) for s in sizes]
    m = max(sz) if sz else 0
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    pad[: t.shape[0]] = t
    if dst is None:
        out = torch.empty((m * ctx.world_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        if dev.type == "cuda":
            dist.all_gather_into_tensor(out, pad, group=group)
        else:
            parts = [torch.empty_like(pad) for _ in range(ctx.world_size)]
            dist.all_gather(parts, pad, group=group)
            out = torch.cat(parts)
    else:
        parts = [torch.empty_like(pad) for _ in range(ctx.world_size)] if ctx.rank == dst else None
        dist.gather(pad, parts, dst=dst, group=group)
        if ctx.rank != dst:
            return None
        out = torch.cat(parts)
    METRICS.inc("dist.bytes_gathered", out.numel() * out.element_size())
    return torch.cat([out[i * m: i * m + s] for i, s in enumerate(sz)])


class GatherSink(SinkFunction):
    def __init__(self, to: Any = "all", lockstep: bool = False, keep: bool = True,
                 on_gathered: Optional[Callable[[np.ndarray, np.ndarray, np.ndarray], None]] = None):
        if to != "all" and to != 0:
            raise ValueError("GatherSink(to=...) must be 'all' or 0")
        self.to = to
        self.lockstep = bool(lockstep)
        self.keep = bool(keep)
        self.on_gathered = on_gathered
        self.dist = None
        self.rows_seen = 0
        self.rows_gathered = 0
        self.gathers = 0
        self._buf: List[Tuple[PredictionBatch, Optional[RecordBatch]]] = []
        self._parts: List[Tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self._comm = None
        self._inflight: List[Any] = []  # (collective works, batches, deliver-on-retire closure)
        self._lock_rows: Optional[int] = None
        self._lock_path: Optional[bool] = None
        self._ring: List[Any] = []
        self._ring_i = 0

    # ------------------------------------------------------------------ lifecycle
    def open(self, context=None) -> None:  # noqa: A003
        self.dist = getattr(context, "dist", None)

    def bind(self, ctx) -> "GatherSink":
        """Use outside a job: attach the :class:`~flink_jpmml_amd.parallel.dist.DistContext`."""
        self.dist = ctx
        return self

    @property
    def _distributed(self) -> bool:
        return self.dist is not None and self.dist.is_distributed

    def invoke(self, value: Any) -> None:
        pb, batch = _split(value)
        self.rows_seen += len(pb)
        if self.lockstep:
            self._gather([(pb, batch)])
        else:
            self._buf.append((pb, batch))

    def pre_commit(self, cid: int) -> None:  # checkpoint barrier / end of input: all ranks meet
        self.flush()
        # retire every in-flight gather before the barrier commits source offsets past its rows:
        # a failure after the commit must not lose rows that were never delivered
        self.finish()

    def commit(self, cid: int) -> None:
        if cid < 0:
            self.finish()

    def close(self) -> None:
        self.finish()

    def flush(self) -> None:
        if self.lockstep:
            return
        buf, self._buf = self._buf, []
        self._gather(buf)

    # ------------------------------------------------------------------ results
    def _deliver(self, s: np.ndarray, v: np.ndarray, o: np.ndarray) -> None:
        v = v.astype(bool, copy=False)
        self.rows_gathered += len(s)
        self.gathers += 1
        if self.keep:
            self._parts.append((s, v, o))
        if self.on_gathered is not None:
            self.on_gathered(s, v, o)

    def _cat(self, i: int, dtype) -> np.ndarray:
        self.finish()
        if not self._parts:
            return np.zeros(0, dtype=dtype)
        return np.concatenate([p[i] for p in self._parts])

    @property
    def scores(self) -> np.ndarray:
        return self._cat(0, np.float32)

    @property
    def valid(self) -> np.ndarray:
        return self._cat(1, bool)

    @property
    def offsets(self) -> np.ndarray:
        return self._cat(2, np.int64)

    # ------------------------------------------------------------------ gathering
    def _gather(self, items: List[Tuple[PredictionBatch, Optional[RecordBatch]]]) -> None:
        import torch

        if not self._distributed:
            for pb, batch in items:
                self._deliver(np.asarray(pb.scores), np.asarray(pb.valid), _row_offsets(pb, batch))
            return
        ctx = self.dist
        device_ok = ctx.backend == "nccl" and items and all(pb.device_out is not None for pb, _ in items)
        if self.lockstep and self._lock_path is not None:
            device_ok = self._lock_path  # decided (collectively) on the first element
        else:
            device_ok = self._agree(bool(device_ok))
            if self.lockstep:
                self._lock_path = device_ok
        if device_ok:
            if self.lockstep:
                self._gather_lockstep_device(items[0])
            else:
                self._gather_device(items)
            return
        g = ctx.group("ctrl")
        s = np.concatenate([np.asarray(pb.scores, dtype=np.float32) for pb, _ in items]) if items else \
            np.zeros(0, np.float32)
        v = np.concatenate([np.asarray(pb.valid, dtype=bool) for pb, _ in items]) if items else np.zeros(0, bool)
        o = np.concatenate([_row_offsets(pb, b) for pb, b in items]) if items else np.zeros(0, np.int64)
        packed = torch.from_numpy(np.stack([s.view(np.int32).astype(np.int64), v.astype(np.int64), o], axis=1)) \
            if len(s) else torch.zeros((0, 3), dtype=torch.int64)
        dst = None if self.to == "all" else 0
        out = gather_varlen(packed, ctx, group=g, dst=dst)
        if out is None:
            return
        a = out.numpy()
        self._deliver(a[:, 0].astype(np.int32).view(np.float32), a[:, 1].astype(bool), a[:, 2].copy())

    def _agree(self, flag: bool) -> bool:
        """Every rank must take the same path (device vs host): logical AND over ranks."""
        from .dist import all_reduce_max

        return not bool(all_reduce_max(0 if flag else 1, self.dist, group=self.dist.group("ctrl")))

    def _stream(self):
        import torch

        if self._comm is None:
            self._comm = torch.cuda.Stream(self.dist.device)
        return self._comm

    def _wait_inputs(self, comm, pbs: List[PredictionBatch]) -> None:
        for pb in pbs:
            ev = getattr(pb, "_done", None)
            if ev is not None:
                comm.wait_event(ev)  # the kernel that writes the mirrors (no host sync)
            for t in pb.device_out:
                t.record_stream(comm)  # the allocator keeps them until the gather has read them

    @staticmethod
    def _h2d(a: np.ndarray, device, keep: list):
        """Stream-ordered copy of a small host array (pinned staging, no host sync); the staging
        tensor goes into ``keep`` so it outlives the copy."""
        import torch

        h = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
        keep.append(h)
        return h.to(device, non_blocking=True)

    @classmethod
    def _masked_mirrors(cls, pb: PredictionBatch, keep: list):
        """The device ``(score, valid)`` mirrors with the per-record size validation applied
        (rows whose vector had the wrong width are EmptyScore on every path, as in
        ``PredictionBatch._finish``). Runs on the current (comm) stream."""
        import torch

        s, v = pb.device_out
        ok = getattr(pb, "_row_ok", None)
        if ok is None or ok.all():
            return s, v
        ok_t = cls._h2d(ok.astype(np.bool_), s.device, keep)
        return torch.where(ok_t, s, torch.full_like(s, float("nan"))), v & ok_t.to(v.dtype)

    def _retire(self, entry) -> None:
        """Complete one in-flight gather: wait for its collective, deliver the rows, then run the
        batches' completion hooks (latency observers) — the kernels finished before the gather."""
        works, pbs, finish = entry
        for w in works:
            w.wait()
        if finish is not None:
            finish()
        for pb in pbs:
            pb.wait()

    def finish(self) -> None:
        """Wait for outstanding asynchronous gathers and move kept results to the host."""
        inflight, self._inflight = self._inflight, []
        for entry in inflight:
            self._retire(entry)

    def _bound_inflight(self, limit: int) -> None:
        while len(self._inflight) >= limit:
            self._retire(self._inflight.pop(0))

    def _gather_device(self, items) -> None:
        """Variable-length device gather without host syncs: the row counts travel on the gloo
        ``ctrl`` group (host integers — the job thread knows them without touching the GPU), the
        payload as one packed byte buffer per rank (scores | valid | source offsets) in a single
        asynchronous RCCL collective on the comm stream. Delivery happens when the gather is
        retired (next flush beyond the in-flight bound, ``finish``, ``close``)."""
        import torch
        import torch.distributed as dist

        from .dist import all_gather_ints

        ctx = self.dist
        pbs = [pb for pb, _ in items]
        n = sum(len(pb) for pb in pbs)
        sizes = all_gather_ints(n, ctx, group=ctx.group("ctrl"))
        m = max(sizes) if sizes else 0
        if m == 0:
            return
        W = ctx.world_size
        row = 13  # float32 score + uint8 valid + int64 source offset
        offs = np.zeros(m, dtype=np.int64)
        if n:
            offs[:n] = np.concatenate([_row_offsets(pb, b) for pb, b in items])
        keep: list = []
        offs_h = torch.from_numpy(offs).pin_memory()
        self._bound_inflight(4)
        comm = self._stream()
        dev = ctx.device
        with torch.cuda.stream(comm):
            self._wait_inputs(comm, pbs)
            buf = torch.zeros(m * row, dtype=torch.uint8, device=dev)
            sv = buf[: 4 * m].view(torch.float32)
            vv = buf[4 * m: 5 * m]
            ov = buf[5 * m:].view(torch.int64)
            k = 0
            for pb in pbs:
                ms, mv = self._masked_mirrors(pb, keep)
                sv[k: k + len(pb)].copy_(ms)
                vv[k: k + len(pb)].copy_(mv.to(torch.uint8))
                k += len(pb)
            ov.copy_(offs_h, non_blocking=True)
            root = self.to == "all" or ctx.rank == 0
            out = torch.empty(W * m * row, dtype=torch.uint8, device=dev) if root else None
            if self.to == "all":
                work = dist.all_gather_into_tensor(out, buf, async_op=True)
            else:
                parts = list(out.chunk(W)) if root else None
                work = dist.gather(buf, parts, dst=0, async_op=True)
            host = torch.empty(W * m * row, dtype=torch.uint8, pin_memory=True) if root else None
        METRICS.inc("dist.bytes_gathered", W * m * row)
        keepalive = (buf, offs_h, out, keep)

        def finish(out=out, host=host, sizes=sizes, m=m, keepalive=keepalive):
            if out is None or not (self.keep or self.on_gathered is not None):
                return
            with torch.cuda.stream(comm):
                host.copy_(out, non_blocking=True)
            comm.synchronize()
            a = host.numpy().reshape(W, m * row)
            s = np.concatenate([a[r, : 4 * m].view(np.float32)[: sizes[r]] for r in range(W)])
            v = np.concatenate([a[r, 4 * m: 5 * m][: sizes[r]] for r in range(W)]).astype(bool)
            o = np.concatenate([a[r, 5 * m:].view(np.int64)[: sizes[r]] for r in range(W)])
            self._deliver(s, v, o)

        self._inflight.append(([work], pbs, finish))

    def _gather_lockstep_device(self, item) -> None:
        """Equal-size per-rank elements: asynchronous ``all_gather_into_tensor`` on the comm stream,
        at most one gather in flight per ring buffer (bounded device memory)."""
        import torch
        import torch.distributed as dist

        pb, batch = item
        n = len(pb)
        if self._lock_rows is None:
            from .dist import all_reduce_max

            lo = -all_reduce_max(-n, self.dist, group=self.dist.group("ctrl"))
            hi = all_reduce_max(n, self.dist, group=self.dist.group("ctrl"))
            if lo != hi:
                raise ValueError(f"GatherSink(lockstep=True) needs equal rows per rank and element ({lo} vs {hi})")
            self._lock_rows = n
            W = self.dist.world_size
            dev = self.dist.device
            self._ring = [(torch.empty(n * W, dtype=torch.float32, device=dev),
                           torch.empty(n * W, dtype=torch.uint8, device=dev)) for _ in range(2)]
        elif n != self._lock_rows:
            raise ValueError("GatherSink(lockstep=True): element row count changed")
        self._bound_inflight(len(self._ring))
        gs, gv = self._ring[self._ring_i]
        self._ring_i = (self._ring_i + 1) % len(self._ring)
        comm = self._stream()
        keep: list = []
        with torch.cuda.stream(comm):
            self._wait_inputs(comm, [pb])
            ms, mv = self._masked_mirrors(pb, keep)
            w1 = dist.all_gather_into_tensor(gs, ms, async_op=True)
            w2 = dist.all_gather_into_tensor(gv, mv.to(torch.uint8) if mv.dtype != torch.uint8 else mv,
                                             async_op=True)
        METRICS.inc("dist.bytes_gathered", gs.numel() * 4 + gv.numel())
        if self.keep or self.on_gathered is not None:
            go = torch.empty(n * self.dist.world_size, dtype=torch.int64, device=gs.device)
            with torch.cuda.stream(comm):
                o = self._h2d(_row_offsets(pb, batch), gs.device, keep)
                w3 = dist.all_gather_into_tensor(go, o, async_op=True)

            def finish(gs=gs, gv=gv, go=go, keep=keep):
                self._deliver(gs.cpu().numpy(), gv.cpu().numpy(), go.cpu().numpy())

            self._inflight.append(([w1, w2, w3], [pb], finish))
        else:
            self._inflight.append(([w1, w2], [pb], lambda keep=keep: None))


__all__ = ["GatherSink", "gather_varlen"]
