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
import mmap
import os
import queue
import socket
import threading
import time
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..api.batch import RecordBatch
from .clock import Clock, current_clock
from .functions import SourceContext, SourceFunction

logger = logging.getLogger(__name__)

_EOS = object()


class CollectionSource(SourceFunction):
    """A finite, replayable sequence (``from_collection``)."""

    chunkable = True

    def __init__(self, items: Iterable[Any]):
        self.items = list(items)

    def iterate(self) -> Iterator[Any]:
        return iter(self.items)

    def seek(self, offset: int) -> Iterator[Any]:
        return iter(self.items[offset:])

    def iterate_shard(self, rank: int, world: int, start: int = 0) -> Iterator[Tuple[int, Any]]:
        """This rank's elements (global offset ``g % world == rank``, ``g >= start``) only."""
        first = start + ((rank - start) % world)
        for g in range(first, len(self.items), world):
            yield g, self.items[g]

    def global_length(self) -> int:
        return len(self.items)

    def read_chunks(self, rank: int, world: int, start: int, size: int) -> Iterator[list]:
        """``(global_offset, element)`` pairs of this rank in lists of ``size`` (C-speed slicing:
        the chunked per-record path)."""
        items = self.items
        first = start + ((rank - start) % world)
        step = size * world
        for a in range(first, len(items), step):
            b = min(len(items), a + step)
            yield list(zip(range(a, b, world), items[a:b:world]))

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

    chunkable = True

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

    def _is_matrix(self) -> bool:
        return hasattr(self.data, "shape") and len(getattr(self.data, "shape", ())) == 2

    def global_length(self) -> int:
        n = int(self.data.shape[0])
        step = int(self.batch_rows or n) or 1
        return self.repeat * ((n + step - 1) // step)

    def iterate_shard(self, rank: int, world: int, start: int = 0) -> Iterator[Tuple[int, RecordBatch]]:
        """Rank-local slices of a matrix source: batch ``g`` belongs to rank ``g % world``; only
        this rank's batches are cut (views, no copies). Iterables fall back to filtering."""
        if not self._is_matrix():
            for g, b in enumerate(self.iterate()):
                if g >= start and g % world == rank:
                    yield g, b
            return
        X = self.data
        n = int(X.shape[0])
        step = int(self.batch_rows or n) or 1
        per = (n + step - 1) // step
        first = start + ((rank - start) % world)
        for g in range(first, self.global_length(), world):
            rep, k = divmod(g, per)
            s = k * step
            yield g, RecordBatch(X[s:s + step], model_id=self.model_id, offset=rep * n + s)

    def iterate(self) -> Iterator[RecordBatch]:
        if self._is_matrix():
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
    header); categorical tokens get the model's PMML codes, missing tokens become NaN.

    ``parse="device"`` (or ``"auto"`` on a GPU box, when every used field is numeric) moves the raw
    bytes to the GPU and parses them there (:mod:`~flink_jpmml_amd.stream.device_text`): batches
    are then device-resident, ``device_chunk_bytes`` of text each, bit-identical to the host
    parser."""

    chunkable = False  # each batch is a large parse: hand it downstream as soon as it exists

    def __init__(self, path: str, model: Any, batch_rows: int = 1 << 16, delimiter: str = ",",
                 columns: Optional[Sequence[str]] = None, threads: int = 0, model_id: Optional[str] = None,
                 chunk_bytes: int = 16 << 20, use_mmap: bool = True, parse: str = "auto", device: Any = None,
                 device_chunk_bytes: int = 64 << 20):
        if parse not in ("auto", "host", "device"):
            raise ValueError(f"parse must be auto / host / device, not {parse!r}")
        self.parse = parse
        self.device = device
        self.device_chunk_bytes = int(device_chunk_bytes)
        self.path = path
        self.model = model  # CompiledPmml, PmmlModel or ModelReader / path
        self.batch_rows = int(batch_rows)
        self.delimiter = delimiter
        self.columns = list(columns) if columns is not None else None
        self.threads = threads
        self.model_id = model_id
        self.chunk_bytes = int(chunk_bytes)
        self.use_mmap = bool(use_mmap)  # parse regular files where they lie (read-window loop otherwise)

    def _compiled(self):
        from ..runtime.compiled import CompiledPmml

        m = self.model
        if hasattr(m, "active_fields") and hasattr(m, "schema"):
            return m
        if hasattr(m, "compiled"):
            return m.compiled
        return CompiledPmml.load(getattr(m, "source_path", m))

    _rank = 0
    _world = 1
    bytes_parsed = 0

    def open_subtask(self, rank: int, world: int) -> None:
        """Rank-local split: this rank parses only the lines that *start* in its
        ``1/world`` byte range of the data section — every input byte is parsed by exactly one
        rank, and no rank reads the others' lines."""
        self._rank, self._world = int(rank), int(world)

    def _device_for_parse(self, compiled, cols):
        """The GPU to parse on, or None (host parser)."""
        if self.parse == "host":
            return None
        import torch

        from .. import native
        from .device_text import device_parse_supported

        if not torch.cuda.is_available():
            if self.parse == "device":
                raise RuntimeError("TextBatchSource(parse='device') needs a GPU")
            return None
        why = device_parse_supported(compiled, cols, native.DEFAULT_MISSING)
        if why is not None:
            if self.parse == "device":
                raise ValueError(f"TextBatchSource(parse='device'): {why}")
            return None
        dev = self.device if self.device is not None else f"cuda:{torch.cuda.current_device()}"
        return torch.device(dev)

    def _line_start_at_or_after(self, fh, p: int, data_start: int) -> int:
        if p <= data_start:
            return data_start
        fh.seek(p - 1)
        return p - 1 + len(fh.readline())

    def iterate(self) -> Iterator[RecordBatch]:
        from .. import native
        from ..utils.metrics import METRICS

        compiled = self._compiled()
        F = compiled.n_features
        self.bytes_parsed = 0
        with open(self.path, "rb") as fh:
            size = os.fstat(fh.fileno()).st_size
            cols = self.columns
            data_start = 0
            if cols is None:
                head = fh.readline()
                data_start = len(head)
                cols = [h.strip().strip('"') for h in head.decode(errors="replace").strip().split(self.delimiter)]
            span = size - data_start
            lo = self._line_start_at_or_after(fh, data_start + span * self._rank // self._world, data_start)
            hi = self._line_start_at_or_after(fh, data_start + span * (self._rank + 1) // self._world, data_start)
            dev = self._device_for_parse(compiled, cols)
            if dev is not None:
                from .device_text import DeviceTextReader

                reader = DeviceTextReader(self.path, compiled, cols, lo, hi, dev, delimiter=self.delimiter,
                                          chunk_bytes=self.device_chunk_bytes, threads=self.threads or 8,
                                          model_id=self.model_id)
                for b in reader:
                    self.bytes_parsed = reader.bytes_read
                    yield b
                METRICS.inc("ingest.bytes_parsed", reader.bytes_read)
                return
            parser = native.RecordParser(compiled, cols, delimiter=self.delimiter, threads=self.threads)
            if hi > lo and self.use_mmap:
                try:
                    mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
                except (OSError, ValueError):
                    mm = None
                if mm is not None:
                    try:
                        yield from self._iterate_mapped(mm, lo, hi, parser, F)
                    finally:
                        mm.close()
                    return
            fh.seek(lo)
            left = hi - lo
            # one reusable read window (no per-chunk bytes concatenation): the unparsed tail of a
            # chunk (a partial line) moves to the front, the next read lands behind it; batches
            # are filled to ``batch_rows`` rows across chunks, so a pinned batch buffer is never
            # handed downstream a few percent full
            buf = bytearray(self.chunk_bytes)
            view = memoryview(buf)
            n_valid = 0
            row = 0
            eof = left <= 0
            rb, filled = None, 0
            while True:
                if not eof and n_valid < len(buf):
                    k = fh.readinto(view[n_valid: n_valid + min(len(buf) - n_valid, left)])
                    left -= k
                    n_valid += k
                    eof = k == 0 or left <= 0
                if eof and n_valid and buf[n_valid - 1] != 0x0A:  # final line without its newline
                    if n_valid == len(buf):
                        view.release()
                        buf.extend(b"\n")
                        view = memoryview(buf)
                    else:
                        buf[n_valid] = 0x0A
                    n_valid += 1
                if rb is None:
                    rb, filled = RecordBatch.pinned(self.batch_rows, F), 0
                used = 0
                if n_valid:
                    m, used = parser.parse(buf, out=rb.X.numpy()[filled:], max_rows=self.batch_rows - filled,
                                           length=n_valid)
                    filled += len(m)
                    self.bytes_parsed += used
                    METRICS.inc("ingest.bytes_parsed", used)
                    if used:
                        tail = bytes(view[used:n_valid])  # the partial line (short)
                        buf[: len(tail)] = tail
                        n_valid -= used
                done = eof and n_valid == 0
                if filled and (filled == self.batch_rows or done):
                    yield RecordBatch(rb.X[:filled], model_id=self.model_id, offset=row)
                    row += filled
                    rb, filled = None, 0
                if done:
                    break
                if not used and (eof or n_valid == len(buf)):
                    if eof:  # unparsable remainder
                        break
                    view.release()
                    buf.extend(bytes(len(buf)))  # a line longer than the window: grow it
                    view = memoryview(buf)
            view.release()


    def _iterate_mapped(self, mm, lo: int, hi: int, parser, F: int) -> Iterator[RecordBatch]:
        """Parse the rank's byte range [lo, hi) where it lies in the page cache (the file is
        memory-mapped: no read() copy, the parser threads fault the pages in in parallel)."""
        from ..utils.metrics import METRICS

        try:
            mm.madvise(mmap.MADV_SEQUENTIAL)
        except (AttributeError, OSError, ValueError):
            pass
        base = np.frombuffer(mm, dtype=np.uint8)  # read-only view: its address, no copy
        try:
            addr0 = base.ctypes.data
            window = max(64, self.chunk_bytes)
            pos, row = lo, 0
            rb, filled = None, 0
            while pos < hi:
                if rb is None:
                    rb, filled = RecordBatch.pinned(self.batch_rows, F), 0
                n = min(hi - pos, window)
                out = rb.X.numpy()[filled:]
                m, used = parser.parse_address(addr0 + pos, n, out, max_rows=self.batch_rows - filled)
                if used == 0:
                    if pos + n < hi:
                        window *= 2  # a line longer than the window
                        continue
                    # the file's last line has no newline: parse a terminated copy of it
                    m, used = parser.parse(bytes(mm[pos:hi]) + b"\n", out=out, max_rows=self.batch_rows - filled)
                    used = hi - pos if used else 0
                    if not used:
                        break
                filled += len(m)
                pos += used
                self.bytes_parsed += used
                METRICS.inc("ingest.bytes_parsed", used)
                if filled == self.batch_rows or pos >= hi:
                    if filled:
                        yield RecordBatch(rb.X[:filled], model_id=self.model_id, offset=row)
                        row += filled
                    rb, filled = None, 0
        finally:
            del base


class ThreadedSource(SourceFunction):
    """Runs a push-style ``SourceFunction.run(ctx)`` (which may block / sleep forever) on its own
    thread; the job thread pulls its elements through a bounded queue, firing timers while it
    waits (so latency-bound micro-batches flush between slow records)."""

    live = True

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
    broadcast to all ranks; all ranks then see the same sequence. Replication runs
    on a background pump thread per rank, on the dedicated ``replicate`` process group — no other
    thread issues collectives on it, so they cannot interleave with the job thread's checkpoint
    collectives on ``ctrl``. ``start`` is where the leader resumes after a restore."""

    live = True

    def __init__(self, inner: Any, ctx=None):
        self.inner = inner
        self.ctx = ctx

    def cancel(self) -> None:
        cancel = getattr(self.inner, "cancel", None)
        if callable(cancel):
            cancel()

    def iterate(self, clock: Optional[Clock] = None, start: int = 0) -> Iterator[Any]:
        from ..parallel.dist import broadcast_object

        ctx = self.ctx
        if ctx is None or not ctx.is_distributed:
            yield from iter_source(self.inner, clock, start)
            return
        clock = clock or current_clock()
        q: "queue.Queue" = queue.Queue(1024)
        err: List[BaseException] = []
        group = ctx.group("replicate")

        def pump():
            try:
                it = iter_source(self.inner, None, start) if ctx.is_root else None
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


class SocketTextSource(SourceFunction):
    """``socketTextStream(host, port)`` (the reference's control stream,
    `E/CheckpointEvaluate.scala:80-82`): one element per delimited line, read **live** as the
    lines arrive (never to EOF first). ``max_retry`` reconnects (with ``retry_delay_s``) when
    the connection cannot be opened or drops, like Flink's ``SocketTextStreamFunction``; the
    stream ends when the peer closes and no retry is left. Under ``torchrun`` the environment
    reads it on rank 0 and replicates the lines (leader mode)."""

    live = True

    def __init__(self, host: str, port: int, delimiter: str = "\n", max_retry: int = 0,
                 retry_delay_s: float = 0.5, connect_timeout_s: float = 10.0):
        self.host = host
        self.port = int(port)
        self.delimiter = delimiter
        self.max_retry = int(max_retry)
        self.retry_delay_s = float(retry_delay_s)
        self.connect_timeout_s = float(connect_timeout_s)
        self._running = True
        self._sock: Optional[socket.socket] = None

    def cancel(self) -> None:
        self._running = False
        s = self._sock
        if s is not None:
            try:
                s.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass

    def _connect(self) -> Optional[socket.socket]:
        deadline = time.monotonic() + self.connect_timeout_s
        while self._running:
            try:
                return socket.create_connection((self.host, self.port), timeout=self.connect_timeout_s)
            except OSError:
                if time.monotonic() >= deadline:
                    raise
                time.sleep(0.05)
        return None

    def iterate(self) -> Iterator[str]:
        attempts = 0
        delim = self.delimiter.encode()
        while self._running:
            try:
                s = self._connect()
            except OSError:
                if attempts >= self.max_retry:
                    raise
                attempts += 1
                time.sleep(self.retry_delay_s)
                continue
            if s is None:
                return
            self._sock = s
            s.settimeout(None)
            buf = b""
            try:
                while self._running:
                    try:
                        blk = s.recv(1 << 16)
                    except OSError:
                        blk = b""
                    if not blk:
                        break
                    buf += blk
                    while True:
                        i = buf.find(delim)
                        if i < 0:
                            break
                        line, buf = buf[:i], buf[i + len(delim):]
                        yield line.decode(errors="replace").rstrip("\r")
            finally:
                self._sock = None
                s.close()
            if buf.strip():
                yield buf.decode(errors="replace").rstrip("\r")
            if attempts >= self.max_retry:
                return
            attempts += 1
            time.sleep(self.retry_delay_s)


def iter_source(src: Any, clock: Optional[Clock] = None, offset: int = 0) -> Iterator[Any]:
    """Iterator over a source's elements starting at ``offset`` (seek when supported)."""
    if isinstance(src, ReplicatedSource):
        return src.iterate(clock, offset)
    if isinstance(src, ThreadedSource):
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
    """Reads one source node for subtask ``rank`` of ``world``, tracking the global offset.

    ``shard`` mode is rank-local: sources implementing ``iterate_shard(rank, world, start)`` (the
    collections and columnar matrices here) hand this rank only its own elements — the other
    ranks' elements are never materialised. Other sources are read in full and filtered
    (``source.foreign_elements`` counts what that costs). ``leader_offset`` is where a leader-read
    replicated source resumes (the minimum over ranks); this rank then skips to its own ``offset``.
    """

    def __init__(self, node, rank: int = 0, world: int = 1, clock: Optional[Clock] = None, offset: int = 0,
                 leader_offset: Optional[int] = None, owner_cuts: Optional[List[int]] = None):
        self.node = node
        # restore of a shard-mode checkpoint taken at another world size: global offset g was owned
        # by old rank g % len(cuts), which processed it iff g < cuts[owner]. ``owner_cuts`` is one
        # such cut list or several *layers* of them (a rescale of a rescale: each earlier world's
        # cuts stay in force until every reader has passed them, runtime.py::_skip_layers)
        if owner_cuts and not isinstance(owner_cuts[0], (list, tuple)):
            owner_cuts = [owner_cuts]
        self.skip_layers: List[List[int]] = [[int(c) for c in lay] for lay in (owner_cuts or []) if lay]
        self._cuts = self.skip_layers or None
        self.rank = rank
        self.world = world
        self.mode = node.dist_mode if world > 1 else "all"
        self.offset = int(offset)  # global elements consumed (next element's global index)
        self.l_count = 0  # "either" mode: L elements seen (round-robin key)
        self._strided = False
        self._skip_until = 0
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
        elif self.mode == "shard" and callable(getattr(src, "iterate_shard", None)):
            self._strided = True
            self._it = src.iterate_shard(rank, world, offset)
        elif isinstance(src, ReplicatedSource) and leader_offset is not None and leader_offset < offset:
            self._it = iter_source(src, clock, leader_offset)
            self._skip_until = offset
            self.offset = int(leader_offset)
        else:
            self._it = iter_source(src, clock, offset)

    def chunks(self, size: int) -> Optional[Iterator[list]]:
        """Lists of ``(global_offset, element)`` pairs when the source can cut them itself
        (``read_chunks``), else ``None`` (iterate element-wise)."""
        src = self.node.source
        rc = getattr(src, "read_chunks", None)
        if rc is None or self.mode not in ("all", "shard") or self._skip_until or self._cuts:
            return None
        rank, world = (self.rank, self.world) if self.mode == "shard" else (0, 1)

        def gen():
            for pairs in rc(rank, world, self.offset, size):
                self.offset = pairs[-1][0] + 1
                yield pairs
            total = getattr(src, "global_length", None)
            if callable(total):
                self.offset = max(self.offset, int(total()))

        return gen()

    def _done_before(self, g: int) -> bool:
        """Global element ``g`` was processed before the restore (by its owner in some layer)."""
        for lay in self._cuts:
            if g < lay[g % len(lay)]:
                return True
        return False

    def __iter__(self) -> Iterator[Tuple[int, Any]]:
        cuts = self._cuts
        if self._strided:  # (global offset, element) pairs of this rank only
            for g, x in self._it:
                self.offset = g + 1
                if cuts is not None and self._done_before(g):
                    continue
                yield g, x
            total = getattr(self.node.source, "global_length", None)
            if callable(total):
                self.offset = max(self.offset, int(total()))
            return
        foreign = 0
        try:
            for x in self._it:
                g = self.offset
                self.offset += 1
                if g < self._skip_until:
                    continue
                if cuts is not None and self._done_before(g):
                    continue
                if self.mode == "shard" and g % self.world != self.rank:
                    foreign += 1
                    continue
                if self.mode == "either" and x[0] == "L":
                    keep = self.l_count % self.world == self.rank
                    self.l_count += 1
                    if not keep:
                        continue
                yield g, x
        finally:
            if foreign:
                from ..utils.metrics import METRICS

                METRICS.inc("source.foreign_elements", foreign)


__all__ = ["BatchSource", "CollectionSource", "GeneratorSource", "ReplicatedSource", "SocketTextSource",
           "SourceReader", "TextBatchSource", "ThreadedSource", "iter_source"]
