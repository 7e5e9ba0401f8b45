"""HIP-graph replay of multi-kernel plans for small micro-batches.

A plan whose ``launch`` enqueues many kernels (segmented ensembles: one plan per segment, device
predicates and tensor-op aggregation; the library-GEMM SVM and MLP plans: torch ops) pays one
launch latency per kernel. For small batches — the latency path of a streaming job — that is a
large part of the time, and its jitter is the p99. :class:`GraphLauncher` captures the plan once
per row bucket (256, 512, …, ``max_rows``) into a HIP graph over static device buffers and
replays it: rows are copied into the bucket's input buffer, the graph runs every kernel of the
plan in one submission, the first ``n`` scores / validity bytes are copied out (to device
tensors, device mirrors, or zero-copy host pointers). Padding rows carry whatever the buffer held
and their outputs are never read.

Measured through the public ``model.predict(RecordBatch)`` path (``profiles/r3ag/``): a segmented
ensemble (5 tree segments, median, device predicates and tensor-op aggregation: dozens of small
launches) p50 1348 → 491 µs at 256 rows and 1009 → 487 µs at 4096 rows, p99 1853 → 619 µs. A
plan of a few large kernels gains nothing and pays the graph's extra copies: the wide MLP
(input staging + 3 GEMMs + output layer) 150 → 155 µs, the tree walk + split reduce
(``profiles/r3x/``) — neither is graphed.

Plans opt in with ``graph_small_batches = True``; the engine routes micro-batches of at most
``max_rows`` rows through the launcher (``ScoringConfig(graph_max_rows=…)``, 0 = off).
"""

from __future__ import annotations

import logging
import threading
from typing import Dict, Optional

logger = logging.getLogger(__name__)

MIN_BUCKET = 256


class GraphLauncher:
    def __init__(self, plan, max_rows: int = 16384):
        self.plan = plan
        self.device = plan.device
        self.max_rows = int(max_rows)
        self._graphs: Dict[int, tuple] = {}
        self._failed = False
        self._lock = threading.Lock()
        self.replays = 0
        from ..ops import _lib

        self._lib = _lib.load()

    @staticmethod
    def bucket(n: int) -> int:
        b = MIN_BUCKET
        while b < n:
            b *= 2
        return b

    def applies(self, n: int, kw: dict) -> bool:
        """Graph path for this launch: a small batch and no outputs beyond score / valid (and
        their device mirrors)."""
        extra = {k for k, v in kw.items() if v is not None}
        return not self._failed and 0 < n <= self.max_rows and extra <= {"score2", "valid2"}

    def _capture(self, b: int, stream):
        import torch

        F = self.plan.n_features
        Xs = torch.zeros((b, F), dtype=torch.float32, device=self.device)
        ss = torch.empty(b, dtype=torch.float32, device=self.device)
        vs = torch.empty(b, dtype=torch.uint8, device=self.device)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            self.plan.launch(Xs, ss, vs, stream=side)  # warm-up: lazy buffers, kernel attributes
            side.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                self.plan.launch(Xs, ss, vs, stream=side)
        side.synchronize()
        return g, Xs, ss, vs

    def _copy(self, dst, src_ptr: int, nbytes: int, stream) -> None:
        from .plans import _addr

        rc = self._lib.pmml_memcpy_async(_addr(dst), src_ptr, nbytes, 4, stream.cuda_stream)  # hipMemcpyDefault
        if rc != 0:
            raise RuntimeError(f"hipMemcpyAsync failed ({rc})")

    def launch(self, X, score, valid, stream=None, score2=None, valid2=None) -> None:
        """Score the ``n`` rows of device matrix ``X`` into ``score`` / ``valid`` (tensors or raw
        device-visible addresses) on ``stream`` by replaying the bucket's graph."""
        import torch

        stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        n = int(X.shape[0])
        b = self.bucket(n)
        entry = self._graphs.get(b)
        if entry is None:
            with self._lock:
                entry = self._graphs.get(b)
                if entry is None:
                    try:
                        entry = self._capture(b, stream)
                    except Exception as e:  # noqa: BLE001 - capture unsupported: eager from now on
                        logger.warning("HIP graph capture of %s failed (%s); launching eagerly",
                                       type(self.plan).__name__, e)
                        self._failed = True
                        self.plan.launch(X, score, valid, stream=stream, score2=score2, valid2=valid2)
                        return
                    self._graphs[b] = entry
        g, Xs, ss, vs = entry
        F = self.plan.n_features
        if not X.is_contiguous() or X.shape[1] != F:
            X = X.contiguous()
        self._copy(Xs, X.data_ptr(), n * F * 4, stream)
        with torch.cuda.stream(stream):
            g.replay()
        for dst, src, width in ((score, ss, 4), (valid, vs, 1), (score2, ss, 4), (valid2, vs, 1)):
            if dst is not None:
                self._copy(dst, src.data_ptr(), n * width, stream)
        self.replays += 1


__all__ = ["GraphLauncher", "MIN_BUCKET"]
