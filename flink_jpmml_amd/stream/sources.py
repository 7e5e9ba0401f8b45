"""Sources of the stream runtime: collections, generators, thread-backed ``run(ctx)`` sources,
columnar RecordBatch sources (incl. one on the native C++ text ingest) and leader-read sources
replicated to every rank.

Every source is read through a :class:`SourceReader`, which numbers elements with a **global
offset** (the element's position in the logical stream). Offsets are what checkpoints record
(`S/api/functions/EvaluationCoFunction.scala:76-96` keeps only metadata; Flink itself restores
source positions — `E/CheckpointEvaluate.scala:53` runs EXACTLY_ONCE) and what a restored job seeks
to. Under data parallelism (one process per GPU, ``torchrun``) the reader also decides which
elements this rank sees:

* ``shard``     — round-robin by global offset: rank ``r`` of ``W`` takes ``g % W == r``
  (the Flink ``rebalance`` of a parallelism-1 source into N subtasks);
* ``replicate`` — every rank reads every element (a ``broadcast`` stream, e.g. control);
* ``either``    — a tagged ``("L", event) / ("R", control)`` sequence: ``R`` replicated, ``L``
  sharded (the deterministic two-input test harness, `T/utils/FlinkTestKits.scala:44-55`);
* ``parallel``  — every rank runs its own instance (``open_subtask(rank, world)``), like a Flink
  source with parallelism N (synthetic generators, per-rank files).
"""

from __future__ import annotations

import itertools
import logging
import queue
import threading
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..api.batch import RecordBatch
from .clock import Clock, current_clock
from .functions import SourceContext, SourceFunction

logger = logging.getLogger(__name__)

_EOS = object()


class CollectionSource(SourceFunction):
    """A finite, replayable sequence (``from_collection``)."""

    def __init__(self, items: Iterable[Any]):
        self.items = list(items)

    def iterate(self) -> Iterator[Any]:
        return iter(self.items)

    def seek(self, offset: int) -> Iterator[Any]:
        return iter(self.items[offset:])

    def __len__(self) -> int:
        return len(self.items)


class GeneratorSource(SourceFunction):
    """Wraps a zero-argument callable returning a fresh iterator (replayable by re-running it)."""

    def __init__(self, factory: Callable[[], Iterable[Any]]):
        self.factory = factory

    def iterate(self) -> Iterator[Any]:
        return iter(self.factory())


class BatchSource(SourceFunction):
    """Columnar source: a ``[rows, F]`` matrix (numpy or torch, pinned preferred) cut into
    RecordBatches of ``batch_rows``, or an iterable of matrices / RecordBatches. ``repeat``
    replays the matrix that many times (synthetic streams). Seekable by batch index."""

    def __init__(self, data: Any, batch_rows: Optional[int] = None, repeat: int = 1,
                 model_id: Optional[str] = None):
        self.data = data
        self.batch_rows = batch_rows
        self.repeat = int(repeat)
        self.model_id = model_id

    def _matrix_batches(self) -> Iterator[RecordBatch]:
        X = self.data
        n = int(X.shape[0])
        step = int(self.batch_rows or n)
        row = 0
        for _ in range(self.repeat):
            for s in range(0, n, step):
                yield RecordBatch(X[s:s + step], model_id=self.model_id, offset=row)
                row += min(step, n - s)

    def iterate(self) -> Iterator[RecordBatch]:
        if hasattr(self.data, "shape") and len(getattr(self.data, "shape", ())) == 2:
            return self._matrix_batches()

        def gen():
            row = 0
            for x in self.data:
                b = x if isinstance(x, RecordBatch) else RecordBatch(x, model_id=self.model_id, offset=row)
                row += len(b)
                yield b
        return gen()


class TextBatchSource(SourceFunction):
    """Delimited text records → RecordBatches in pinned memory, parsed by the native multi-threaded
    C++ ingest (:class:`flink_jpmml_amd.native.RecordParser`) straight into the batch buffer.
    Columns are matched to the model's active fields by header name (``columns`` overrides the
    header); categorical tokens get the model's PMML codes, missing tokens become NaN."""

    def __init__(self, path: str, model: Any, batch_rows: int = 1 << 16, delimiter: str = ",",
                 columns: Optional[Sequence[str]] = None, threads: int = 0, model_id: Optional[str] = None,
                 chunk_bytes: int = 16 << 20):
        self.path = path
        self.model = model  # CompiledPmml, PmmlModel or ModelReader / path
        self.batch_rows = int(batch_rows)
        self.delimiter = delimiter
        self.columns = list(columns) if columns is not None else None
        self.threads = threads
        self.model_id = model_id
        self.chunk_bytes = int(chunk_bytes)

    def _compiled(self):
        from ..runtime.compiled import CompiledPmml

        m = self.model
        if hasattr(m, "active_fields") and hasattr(m, "schema"):
            return m
        if hasattr(m, "compiled"):
            return m.compiled
        return CompiledPmml.load(getattr(m, "source_path", m))

    def iterate(self) -> Iterator[RecordBatch]:
        from .. import native

        compiled = self._compiled()
        F = compiled.n_features
        with open(self.path, "rb") as fh:
            head = fh.readline()
            cols = self.columns
            if cols is None:
                cols = [h.strip().strip('"') for h in head.decode(errors="replace").strip().split(self.delimiter)]
            else:
                fh.seek(0)
            parser = native.RecordParser(compiled, cols, delimiter=self.delimiter, threads=self.threads)
            rest = b""
            row = 0
            eof = False
            while not eof or rest:
                if not eof and len(rest) < self.chunk_bytes:
                    blk = fh.read(self.chunk_bytes)
                    eof = not blk
                    rest += blk
                    if eof and rest and not rest.endswith(b"\n"):
                        rest += b"\n"
                    if not eof:
                        continue
                if not rest:
                    break
                rb = RecordBatch.pinned(self.batch_rows, F)
                m, used = parser.parse(rest, out=rb.X.numpy(), max_rows=self.batch_rows)
                if used == 0:
                    break
                rest = rest[used:]
                rb = RecordBatch(rb.X[: len(m)], model_id=self.model_id, offset=row)
                row += len(m)
                if len(m):
                    yield rb


class ThreadedSource(SourceFunction):
    """Runs a push-style ``SourceFunction.run(ctx)`` (which may block / sleep forever) on its own
    thread; the job thread pulls its elements through a bounded queue, firing timers while it
    waits (so latency-bound micro-batches flush between slow records)."""

    def __init__(self, inner: SourceFunction, capacity: int = 1024):
        self.inner = inner
        self.capacity = capacity

    def iterate(self, clock: Optional[Clock] = None) -> Iterator[Any]:
        clock = clock or current_clock()
        q: "queue.Queue" = queue.Queue(self.capacity)
        err: List[BaseException] = []

        def run():
            try:
                self.inner.run(SourceContext(q.put, threading.Lock()))
            except BaseException as e:  # noqa: BLE001 - re-raised on the job thread
                err.append(e)
            finally:
                q.put(_EOS)

        t = threading.Thread(target=run, name=f"source-{type(self.inner).__name__}", daemon=True)
        t.start()
        try:
            while True:
                x = clock.get(q)
                if x is _EOS:
                    if err:
                        raise err[0]
                    return
                yield x
        finally:
            self.inner.cancel()


class ReplicatedSource(SourceFunction):
    """A source only rank 0 can read (a socket, a queue): rank 0 iterates it and every element is
    broadcast to all ranks on the control process group; all ranks then see the
    same sequence. Replication runs on a background thread per rank."""

    def __init__(self, inner: Any, ctx=None):
        self.inner = inner
        self.ctx = ctx

    def iterate(self, clock: Optional[Clock] = None) -> Iterator[Any]:
        from ..parallel.dist import broadcast_object

        ctx = self.ctx
        if ctx is None or not ctx.is_distributed:
            yield from iter_source(self.inner, clock)
            return
        clock = clock or current_clock()
        q: "queue.Queue" = queue.Queue(1024)
        err: List[BaseException] = []
        group = ctx.group("ctrl")

        def pump():
            try:
                it = iter_source(self.inner, None) if ctx.is_root else None
                while True:
                    x = None
                    if ctx.is_root:
                        x = next(it, _EOS)
                        x = ("eos",) if x is _EOS else ("x", x)
                    x = broadcast_object(x, ctx, group=group)
                    if x[0] == "eos":
                        return
                    q.put(x[1])
            except BaseException as e:  # noqa: BLE001
                err.append(e)
            finally:
                q.put(_EOS)

        t = threading.Thread(target=pump, name="replicated-source", daemon=True)
        t.start()
        while True:
            x = clock.get(q)
            if x is _EOS:
                if err:
                    raise err[0]
                return
            yield x


def iter_source(src: Any, clock: Optional[Clock] = None, offset: int = 0) -> Iterator[Any]:
    """Iterator over a source's elements starting at ``offset`` (seek when supported)."""
    if isinstance(src, (ThreadedSource, ReplicatedSource)):
        it = src.iterate(clock)
    elif hasattr(src, "seek") and offset:
        return iter(src.seek(offset))
    elif isinstance(src, SourceFunction):
        if type(src).iterate is SourceFunction.iterate:  # push-only source: run it on a thread
            it = ThreadedSource(src).iterate(clock)
        else:
            it = iter(src.iterate())
    elif callable(getattr(src, "iterate", None)):  # duck-typed pull source
        it = iter(src.iterate())
    elif callable(getattr(src, "run", None)) and not hasattr(src, "__iter__"):  # duck-typed push source
        it = ThreadedSource(src).iterate(clock)
    else:
        it = iter(src)
    if offset:
        it = itertools.islice(it, offset, None)
    return it


class SourceReader:
    """Reads one source node for subtask ``rank`` of ``world``, tracking the global offset."""

    def __init__(self, node, rank: int = 0, world: int = 1, clock: Optional[Clock] = None, offset: int = 0):
        self.node = node
        self.rank = rank
        self.world = world
        self.mode = node.dist_mode if world > 1 else "all"
        self.offset = int(offset)  # global elements consumed (next element's global index)
        self.l_count = 0  # "either" mode: L elements seen (round-robin key)
        src = node.source
        if self.mode == "parallel" and hasattr(src, "open_subtask"):
            src.open_subtask(rank, world)
        if self.mode == "either" and offset:
            # the round-robin key of L elements must continue where it stopped: replay the prefix
            self._it = iter_source(src, clock, 0)
            for _ in range(offset):
                tag, _ = next(self._it)
                if tag == "L":
                    self.l_count += 1
        else:
            self._it = iter_source(src, clock, offset)

    def __iter__(self) -> Iterator[Tuple[int, Any]]:
        for x in self._it:
            g = self.offset
            self.offset += 1
            if self.mode == "shard" and g % self.world != self.rank:
                continue
            if self.mode == "either" and x[0] == "L":
                keep = self.l_count % self.world == self.rank
                self.l_count += 1
                if not keep:
                    continue
            yield g, x


__all__ = ["BatchSource", "CollectionSource", "GeneratorSource", "ReplicatedSource", "SourceReader",
           "TextBatchSource", "ThreadedSource", "iter_source"]
