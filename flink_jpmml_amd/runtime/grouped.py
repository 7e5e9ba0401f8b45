"""Mixed-model micro-batches scored in one pass (dynamic serving at columnar speed).

The reference's dynamic operator serves many models from one operator: each event names its
model and ``processElement1`` picks it from the cache (`S/package.scala:107-119`,
`S/api/functions/EvaluationCoFunction.scala:106-117`). A columnar batch here carries one model
code per row (``RecordBatch(model_ids=(codes, keys))``). Splitting such a batch on the host costs a
128-byte row gather per record through host memory and one pageable H2D per model. The
:class:`GroupedScorer` instead moves the batch across PCIe once, in arrival order, and groups it in
HBM (``ops/csrc/grouped.hip``)::

    copy streams:  pinned rows ──▶ ring slot          pinned codes ──▶ code slot
    compute:       group_rows_kernel (rows → per-model contiguous ranges, inverse permutation)
                   ▶ one launch per model present (the model's own plan: tree / NN / ... kernels)
                   ▶ ungroup_kernel: scores back in row order, written zero-copy into pinned host
                     memory (+ optional device mirrors for an all-gather sink)

The host's per-row work is one pass over the codes (the per-model row counts size the launches);
everything else is O(models) per micro-batch. The result is ONE :class:`PredictionBatch` in row
order — row ``i`` equals ``model_for(id_i).predict(batch.vector(i))``.

**Device-counted path** (every model a wide-kernel tree ensemble — the common serving case): the
host does no per-row work at all and issues THREE kernels per slice whatever the number of models::

    group_count_kernel   per-model counts + prefixes on the device (row ranges, tile numbering)
    group_place_kernel   rows -> model-contiguous Xg, perm[pos] = arrival row, EmptyScore rows
    tree_grouped_wide_kernel   ONE launch: workgroup -> (model, tile) through the device tile
                         table, each model's own forest / prepare / epilogue, outputs scattered
                         back to arrival order in HBM (then one D2H copy of the slice's scores)

(one tree launch per distinct kernel configuration — depth, leaf format, tile rows, accumulation
mode — so a fleet of same-shaped models is one launch). Models on other kernels take the
host-counted path above.
"""

from __future__ import annotations

import collections
from typing import List, Optional, Sequence

import numpy as np

from ..api.batch import PredictionBatch, RecordBatch
from ..utils.metrics import METRICS
from ..utils.profiling import prange
from .engine import DevicePipeline, NullScorer, StreamingScorer, _observe_latency, _pin

MAX_GROUP_MODELS = 1024  # group_rows_kernel keeps one LDS counter per model


class NotGroupable(Exception):
    """The batch cannot take the grouped device path (host-scored models, mixed widths, too many
    models); the caller splits it per model instead."""


def groupable(scorers: Sequence[object], width: int) -> Optional[str]:
    """``None`` when every scorer can run in a grouped launch over ``width``-column rows, else the
    reason it cannot."""
    if len(scorers) > MAX_GROUP_MODELS:
        return f"{len(scorers)} models in one batch (max {MAX_GROUP_MODELS})"
    pipe = None
    for s in scorers:
        if isinstance(s, NullScorer):
            continue
        if not isinstance(s, StreamingScorer):
            return f"model scored by {type(s).__name__}"
        if s.F != width:
            return f"model expects {s.F} features, batch has {width}"
        if pipe is None:
            pipe = s.pipe
        elif s.pipe is not pipe:
            return "models on different device pipelines"
    return None


class GroupedScorer:
    """Grouped scoring of mixed-model batches on one :class:`DevicePipeline` (its copy streams and
    compute stream, shared with the per-model scorers of the same operator).

    Slices are sized so each model present gets about ``rows_per_model`` rows per launch (one
    1024-thread workgroup per 256-row tile over the chip's 256 CUs), between the pipeline's
    micro-batch and ``max_slice`` rows; the grouper keeps its own input ring for them. Tree plans
    of the slice launch from ONE host call (``pmml_tree_launch_many``); other plans launch one by
    one."""

    kind = "grouped"

    def __init__(self, pipe: DevicePipeline, max_inflight: int = 4, rows_per_model: int = 1 << 16,
                 max_slice: int = 1 << 23):
        from ..ops import _lib

        self.pipe = pipe
        self.device = pipe.device
        self.B = pipe.B
        self.rows_per_model = int(rows_per_model)
        self.max_slice = int(max_slice)
        self.max_inflight = int(max_inflight)
        self._lib = _lib.load()
        self._S = 0
        self._F = 0
        self._work = None  # (Xg, inv, sg, vg): compute-stream scratch, reused slice after slice
        self._ring: List[dict] = []
        self._next = 0
        self._inflight: "collections.deque" = collections.deque()
        self.rows_submitted = 0
        self._dg: Optional[dict] = None  # device-counted grouping tables of the current scorer set
        self.device_grouping = True

    # ------------------------------------------------------------------ buffers
    def slice_rows(self, n_models: int) -> int:
        return int(min(self.max_slice, max(self.B, n_models * self.rows_per_model)))

    def _ensure(self, S: int, F: int) -> None:
        import torch

        if self._work is not None and self._S >= S and self._F >= F:
            return
        p = self.pipe
        old = list(self._work or ()) + [t for r in self._ring for t in (r["x"], r["codes"])]
        for t in old:  # queued copies / kernels may still use the old buffers
            t.record_stream(p.comp)
            for st in p.h2ds:
                t.record_stream(st)
        dev = self.device
        self._work = (torch.empty(S * F, dtype=torch.float32, device=dev), torch.empty(S, dtype=torch.int32, device=dev),
                      torch.empty(S, dtype=torch.float32, device=dev), torch.empty(S, dtype=torch.uint8, device=dev))
        self._ring = [{"x": torch.empty(S * F, dtype=torch.float32, device=dev),
                       "codes": torch.empty(S * 2, dtype=torch.uint8, device=dev),
                       "ev_h2d": [torch.cuda.Event() for _ in p.h2ds], "ev_comp": torch.cuda.Event(), "used": False}
                      for _ in range(p.depth)]
        self._next = 0
        self._S, self._F = S, F

    def _throttle(self) -> None:
        while len(self._inflight) >= self.max_inflight:
            self._inflight.popleft()[0].synchronize()
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()

    # ------------------------------------------------------------------ scoring
    def submit(self, batch: RecordBatch, codes, scorers: Sequence[object], keep_device: bool = False) -> PredictionBatch:
        """Score ``batch`` whose row ``i`` belongs to ``scorers[codes[i]]`` (``NullScorer`` →
        EmptyScore). Returns the row-order :class:`PredictionBatch` future immediately."""
        import torch

        from ..ops._lib import check

        n = len(batch)
        if n == 0:
            return PredictionBatch.empty(0)
        F = batch.n_features
        K = len(scorers)
        why = groupable(scorers, F)
        if why is not None:
            raise NotGroupable(why)
        p = self.pipe
        lib = self._lib
        # ---- host side: rows and codes in pinned memory
        X = batch.X
        with prange("grouped.stage"):
            if not isinstance(X, torch.Tensor):
                X = _pin(X)
            elif X.is_cuda:
                if X.dtype != torch.float32 or not X.is_contiguous():
                    X = X.to(torch.float32).contiguous()
                if getattr(batch, "ready", None) is not None:
                    p.comp.wait_event(batch.ready)
                else:
                    p.comp.wait_stream(torch.cuda.current_stream(self.device))
                X.record_stream(p.comp)
            elif not X.is_pinned() or X.dtype != torch.float32 or not X.is_contiguous():
                X = _pin(X)
            cdt = torch.uint8 if K <= 256 else torch.int16
            code_bytes = 1 if K <= 256 else 2
            if isinstance(codes, torch.Tensor) and codes.dtype == cdt and codes.is_contiguous() and \
                    (codes.is_pinned() or codes.is_cuda):
                codes_t = codes
            else:
                c_np = codes.numpy() if isinstance(codes, torch.Tensor) else np.asarray(codes)
                if len(c_np) != n or (n and (int(c_np.min()) < 0 or int(c_np.max()) >= K)):
                    raise ValueError(f"model codes must be {n} values in [0, {K})")
                codes_t = torch.empty(n, dtype=cdt, pin_memory=True)
                codes_t.numpy()[:] = c_np
            codes_np = codes_t.cpu().numpy() if codes_t.is_cuda else codes_t.numpy()
            if codes_t is codes:  # pinned / device codes: the same range check as the host path
                # (the device-counted kernels would otherwise answer EmptyScore silently
                # where the host-counted path raises)
                if len(codes_np) != n or (n and not (K >= 256 and cdt == torch.uint8) and (
                        int(codes_np.max()) >= K or (cdt != torch.uint8 and int(codes_np.min()) < 0))):
                    raise ValueError(f"model codes must be {n} values in [0, {K})")
        S = self.slice_rows(K)
        self._ensure(S, F)
        self._throttle()
        Xg, inv, sg, vg = self._work
        score_h = torch.empty(n, dtype=torch.float32, pin_memory=True)
        valid_h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        dg = self._device_tables(scorers, F) if self.device_grouping else None
        if dg is not None:
            return self._submit_device(batch, X, codes_t, code_bytes, n, F, S, dg, score_h, valid_h, keep_device)
        hs, hv = p.host_dev_ptr(score_h), p.host_dev_ptr(valid_h)
        dev_out = None
        if keep_device or hs is None:
            with torch.cuda.stream(p.comp):
                dev_out = (torch.empty(n, dtype=torch.float32, device=self.device),
                           torch.empty(n, dtype=torch.uint8, device=self.device))
        keep = []
        with prange("grouped.enqueue"):
            for s in range(0, n, S):
                e = min(n, s + S)
                m = e - s
                with prange("grouped.count"):
                    counts = np.bincount(codes_np[s:e], minlength=K)
                    if len(counts) > K:
                        raise ValueError(f"model code {len(counts) - 1} out of range [0, {K})")
                    starts = np.zeros(K + 1, dtype=np.int64)
                    np.cumsum(counts, out=starts[1:])
                # ---- H2D of the rows and the codes into the next ring slot
                slot = self._ring[self._next]
                self._next = (self._next + 1) % len(self._ring)
                xs_ptr, ldx, cs_ptr = self._stage(X, codes_t, s, m, F, code_bytes, slot)
                # ---- compute: group, launch every model present, ungroup
                cur_h = torch.from_numpy(starts[:K].astype(np.int32)).pin_memory()
                keep.append(cur_h)
                cursor = self._cursor(K)
                check(lib.pmml_memcpy_async(cursor.data_ptr(), cur_h.data_ptr(), K * 4, 1, p.comp.cuda_stream),
                      "group cursor H2D")
                check(lib.pmml_group_rows(p.comp.cuda_stream, xs_ptr, ldx, F, m, cs_ptr, code_bytes, K,
                                          cursor.data_ptr(), Xg.data_ptr(), inv.data_ptr()), "group_rows kernel")
                with prange("grouped.launch"):
                    self._launch_models(scorers, counts, starts, Xg, sg, vg, F, keep)
                os_ = hs + 4 * s if hs is not None else dev_out[0][s:e].data_ptr()
                ov_ = hv + s if hv is not None else dev_out[1][s:e].data_ptr()
                s2 = dev_out[0][s:e].data_ptr() if (dev_out is not None and hs is not None) else None
                v2 = dev_out[1][s:e].data_ptr() if (dev_out is not None and hs is not None) else None
                check(lib.pmml_ungroup(p.comp.cuda_stream, sg.data_ptr(), vg.data_ptr(), inv.data_ptr(), m, os_, ov_,
                                       s2, v2), "ungroup kernel")
                slot["ev_comp"].record(p.comp)
                slot["used"] = True
                METRICS.inc("grouped.models_launched", int(np.count_nonzero(counts)))
                METRICS.inc("grouped.slices")
            done = torch.cuda.Event()
            if hs is None:
                ev = torch.cuda.Event()
                ev.record(p.comp)
                with torch.cuda.stream(p.d2h):
                    p.d2h.wait_event(ev)
                    score_h.copy_(dev_out[0], non_blocking=True)
                    valid_h.copy_(dev_out[1], non_blocking=True)
                    for t in dev_out:
                        t.record_stream(p.d2h)
                done.record(p.d2h)
            else:
                done.record(p.comp)
        self._inflight.append((done, X, codes_t, keep))
        self.rows_submitted += n
        METRICS.inc("grouped.rows", n)
        METRICS.inc("grouped.batches")
        return PredictionBatch(n, score_h, valid_h, done, owner=(X, codes_t, dev_out, keep),
                               on_done=_observe_latency, device_out=dev_out, row_ok=batch.size_ok())

    # ------------------------------------------------------------------ device-counted path
    def _device_tables(self, scorers, F: int) -> Optional[dict]:
        """Launch tables of the device-counted path for this scorer set (cached while the set is
        unchanged), or ``None`` when some model does not score with the wide tree kernel."""
        import ctypes

        import torch

        from ..ops._lib import TreeArgs

        key = (tuple(id(sc) for sc in scorers), F)
        if self._dg is not None and self._dg["key"] == key:
            return self._dg
        K = len(scorers)
        tile_rows = np.zeros(K, dtype=np.int32)
        groups: dict = {}
        for k, sc in enumerate(scorers):
            if isinstance(sc, NullScorer):
                continue
            fn = getattr(getattr(sc, "plan", None), "grouped_args", None)
            got = fn(F) if fn is not None else None
            if got is None:
                return None
            a, depth, gkey, rows = got
            tile_rows[k] = rows
            groups.setdefault(gkey, []).append((k, a))
        order, launches, args = [], [], []
        for gkey in sorted(groups):
            ents = groups[gkey]
            launches.append(dict(gs=len(order), n=len(ents), depth=gkey[0], rows=gkey[2]))
            order.extend(k for k, _ in ents)
            args.extend(a for _, a in ents)
        dev = self.device
        n_ent = len(order)
        host_arr = (TreeArgs * max(1, n_ent))(*args)
        raw = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(host_arr), ctypes.sizeof(host_arr))),
                               dtype=torch.uint8)
        i32 = dict(dtype=torch.int32, device=dev)
        # the zero-fills of ``counts`` / ``ticket`` (the last-workgroup ticket
        # scheme needs both zero) and the table uploads are enqueued on the compute stream the
        # group kernels run on, so stream order guarantees they land first
        with torch.cuda.stream(self.pipe.comp):
            dg = dict(key=key, scorers=list(scorers), K=K, n_entries=n_ent, launches=launches, host_arr=host_arr,
                      models=raw.to(dev), order=torch.tensor(order or [0], **i32),
                      tile_rows=torch.from_numpy(tile_rows).to(dev), counts=torch.zeros(K, **i32),
                      ticket=torch.zeros(1, **i32), cursor=torch.empty(K, **i32), row_start=torch.empty(K + 1, **i32),
                      tile_start=torch.empty(n_ent + 1, **i32), arg_size=ctypes.sizeof(TreeArgs))
        if self._dg is not None:  # queued kernels may still read the old tables
            for t in (self._dg["models"], self._dg["order"], self._dg["tile_rows"], self._dg["counts"],
                      self._dg["ticket"], self._dg["cursor"], self._dg["row_start"], self._dg["tile_start"]):
                t.record_stream(self.pipe.comp)
        self._dg = dg
        return dg

    def _submit_device(self, batch, X, codes_t, code_bytes: int, n: int, F: int, S: int, dg: dict, score_h, valid_h,
                       keep_device: bool) -> PredictionBatch:
        import ctypes

        import torch

        from ..ops._lib import GroupedTreeArgs, check

        p, lib = self.pipe, self._lib
        Xg, perm = self._work[0], self._work[1]
        with torch.cuda.stream(p.comp):
            dev_out = (torch.empty(n, dtype=torch.float32, device=self.device),
                       torch.empty(n, dtype=torch.uint8, device=self.device))
        K, n_ent = dg["K"], dg["n_entries"]
        cs = p.comp.cuda_stream
        with prange("grouped.enqueue"):
            for s in range(0, n, S):
                e = min(n, s + S)
                m = e - s
                slot = self._ring[self._next]
                self._next = (self._next + 1) % len(self._ring)
                xs_ptr, ldx, cs_ptr = self._stage(X, codes_t, s, m, F, code_bytes, slot)
                out_s, out_v = dev_out[0][s:e].data_ptr(), dev_out[1][s:e].data_ptr()
                check(lib.pmml_group_slice(cs, xs_ptr, ldx, F, m, cs_ptr, code_bytes, K, dg["tile_rows"].data_ptr(),
                                           dg["order"].data_ptr(), n_ent, dg["counts"].data_ptr(),
                                           dg["ticket"].data_ptr(), dg["cursor"].data_ptr(),
                                           dg["row_start"].data_ptr(), dg["tile_start"].data_ptr(), Xg.data_ptr(),
                                           perm.data_ptr(), out_s, out_v), "group count / place kernels")
                for ln in dg["launches"]:
                    gs, cnt = ln["gs"], ln["n"]
                    ga = GroupedTreeArgs(models=dg["models"].data_ptr() + gs * dg["arg_size"],
                                         model_code=dg["order"].data_ptr() + 4 * gs,
                                         row_start=dg["row_start"].data_ptr(),
                                         tile_start=dg["tile_start"].data_ptr() + 4 * gs, Xg=Xg.data_ptr(),
                                         perm=perm.data_ptr(), out_s=out_s, out_v=out_v, n_models=cnt, F=F)
                    tiles = -(-m // ln["rows"]) + cnt
                    rc = lib.pmml_tree_launch_grouped(cs, ctypes.addressof(dg["host_arr"]) + gs * dg["arg_size"], cnt,
                                                      ctypes.byref(ga), ln["depth"], tiles)
                    check(rc, "grouped tree launch")
                slot["ev_comp"].record(p.comp)
                slot["used"] = True
                # this slice's scores back to the host while the next slice is grouped and scored
                with torch.cuda.stream(p.d2h):
                    p.d2h.wait_event(slot["ev_comp"])
                    score_h[s:e].copy_(dev_out[0][s:e], non_blocking=True)
                    valid_h[s:e].copy_(dev_out[1][s:e], non_blocking=True)
                METRICS.inc("grouped.tree_launches", len(dg["launches"]))
                METRICS.inc("grouped.slices")
            for t in dev_out:
                t.record_stream(p.d2h)
            done = torch.cuda.Event()
            done.record(p.d2h)
        keep = [dg["host_arr"]]
        self._inflight.append((done, X, codes_t, keep))
        self.rows_submitted += n
        METRICS.inc("grouped.rows", n)
        METRICS.inc("grouped.batches")
        METRICS.inc("grouped.device_counted_batches")
        return PredictionBatch(n, score_h, valid_h, done, owner=(X, codes_t, dev_out, keep, dg),
                               on_done=_observe_latency, device_out=dev_out if keep_device else None,
                               row_ok=batch.size_ok())

    def _stage(self, X, codes_t, s: int, m: int, F: int, code_bytes: int, slot: dict):
        """Rows ``[s, s + m)`` and their codes on the device (copied into ``slot`` unless already
        there). Returns ``(rows pointer, row stride, codes pointer)``."""
        from ..ops._lib import check

        p, lib = self.pipe, self._lib
        if X.is_cuda and codes_t.is_cuda:
            return X.data_ptr() + s * X.stride(0) * 4, X.stride(0), codes_t.data_ptr() + s * code_bytes
        h2ds = p.active_h2d()
        if len(h2ds) > 1 and m * F * 4 < (8 << 20):
            h2ds = h2ds[:1]
        for st in h2ds:
            if slot["used"]:
                st.wait_event(slot["ev_comp"])  # the kernels of this slot's last use are done
        if X.is_cuda:
            x_ptr, ldx = X.data_ptr() + s * X.stride(0) * 4, X.stride(0)
        else:
            x_ptr, ldx = slot["x"].data_ptr(), F
            part = -(-m // len(h2ds))
            rowb = F * 4
            for j, st in enumerate(h2ds):
                a, b = j * part, min(m, (j + 1) * part)
                if a < b:
                    check(lib.pmml_memcpy_async(x_ptr + a * rowb, X.data_ptr() + (s + a) * rowb, (b - a) * rowb, 1,
                                                st.cuda_stream), "rows H2D")
        if codes_t.is_cuda:
            c_ptr = codes_t.data_ptr() + s * code_bytes
        else:
            c_ptr = slot["codes"].data_ptr()
            check(lib.pmml_memcpy_async(c_ptr, codes_t.data_ptr() + s * code_bytes, m * code_bytes, 1,
                                        h2ds[0].cuda_stream), "codes H2D")
        for j, st in enumerate(h2ds):
            slot["ev_h2d"][j].record(st)
            p.comp.wait_event(slot["ev_h2d"][j])
        return x_ptr, ldx, c_ptr

    def _launch_models(self, scorers, counts, starts, Xg, sg, vg, F: int, keep: list) -> None:
        """One launch per model present in the slice: tree plans batched into one native call."""
        import ctypes

        import torch

        from ..ops._lib import TreeArgs, check

        p = self.pipe
        args, meta = [], []
        with torch.cuda.stream(p.comp):
            for k in np.flatnonzero(counts).tolist():
                a, b = int(starts[k]), int(starts[k + 1])
                sc = scorers[k]
                if not isinstance(sc, StreamingScorer):  # NullScorer: EmptyScore rows
                    vg[a:b].zero_()
                    sg[a:b].fill_(float("nan"))
                    continue
                la = getattr(sc.plan, "batch_launch_args", None)
                got = la(Xg.data_ptr() + a * F * 4, b - a, F, F, sg.data_ptr() + 4 * a, vg.data_ptr() + a) \
                    if la is not None else None
                if got is None:
                    sc.plan.launch(Xg[a * F: b * F].view(b - a, F), sg[a:b], vg[a:b], stream=p.comp)
                else:
                    args.append(got[0])
                    meta.extend(got[1])
        if args:
            arr = (TreeArgs * len(args))(*args)
            mt = (ctypes.c_int * len(meta))(*meta)
            keep.append((arr, mt))
            rc = self._lib.pmml_tree_launch_many(p.comp.cuda_stream, ctypes.cast(arr, ctypes.c_void_p),
                                                 ctypes.cast(mt, ctypes.c_void_p), len(args))
            check(rc, f"grouped tree launches (launch {rc >> 8})")

    def _cursor(self, K: int):
        import torch

        c = getattr(self, "_cursor_buf", None)
        if c is None or c.numel() < K:
            if c is not None:
                c.record_stream(self.pipe.comp)
            c = self._cursor_buf = torch.empty(max(K, 256), dtype=torch.int32, device=self.device)
        return c

    def drain(self) -> None:
        while self._inflight:
            self._inflight.popleft()[0].synchronize()


__all__ = ["GroupedScorer", "MAX_GROUP_MODELS", "NotGroupable", "groupable"]
