"""Input multiplexing of the job thread: how the elements of several sources reach the operators.

The reference runs on Flink, where every source is its own task thread and an operator with two
inputs processes whichever input has data (`S/package.scala:65,118`: events keep flowing while the
broadcast control stream is idle for seconds, `E/CheckpointEvaluate.scala:56-82`,
`E/DynamicEvaluateKmeans.scala:50-60`). Two multiplexers implement that here:

* :class:`LiveInputs` — **available-first**. One reader thread per source pulls its iterator (which
  may block in a socket read or sleep between records) and hands elements to one FIFO; the job
  thread takes whatever arrived first, firing processing-time timers while it waits. An idle
  source never delays another source's elements. Backpressure is a bounded number of queued
  chunks per source. Checkpoint barriers and the end-of-job stop are :class:`Marker`s put into the
  same FIFO from any thread: everything enqueued before a barrier is processed before it, so the
  per-source *processed* counts at the barrier are an exact cut (Flink's aligned checkpoint of a
  single-channel input).
* :class:`DeterministicInputs` — the reproducible merge for bounded, non-blocking sources and
  test harnesses: by timestamp when every source defines one (the analogue of
  `T/sources/TemporizedSourceFunction.scala:35-56`), else round-robin. Used with a
  :class:`~flink_jpmml_amd.stream.clock.ManualClock` (virtual time lives on the job thread).

Both yield ``(node, global_offset, element)`` triples, :class:`Marker`s and (live only)
:data:`IDLE` wake-ups when nothing arrived within the poll period (watchdog kicks, time-based
checkpoint checks).
"""

from __future__ import annotations

import heapq
import itertools
import queue
import threading
from typing import Any, Iterator, List, Optional

from ..utils.metrics import METRICS
from .clock import Clock, set_current_clock

_seq = itertools.count()


class Marker:
    """In-band control item of the job's input FIFO: ``barrier`` (checkpoint ``cid``), ``stop``
    (distributed end of job), ``error`` (a coordinator failure to raise on the job thread)."""

    __slots__ = ("kind", "cid", "exc")

    def __init__(self, kind: str, cid: int = 0, exc: Optional[BaseException] = None):
        self.kind = kind
        self.cid = int(cid)
        self.exc = exc

    def __repr__(self) -> str:
        return f"Marker({self.kind}, cid={self.cid})"


IDLE = Marker("idle")


class Chunk:
    """Several consecutive ``(global_offset, element)`` pairs of one source, delivered downstream
    with one ``collect_many`` (amortises the per-element dispatch of per-record streams)."""

    __slots__ = ("node", "pairs")

    def __init__(self, node: Any, pairs: list):
        self.node = node
        self.pairs = pairs


def is_chunkable_source(src: Any) -> bool:
    """Sources whose reads never block or sleep (in-memory collections, columnar matrices, files):
    the deterministic merge may pull several elements ahead and deliver them as one chunk."""
    return bool(getattr(src, "chunkable", False)) and not is_live_source(src)


class _Eos:
    __slots__ = ("si",)

    def __init__(self, si: int):
        self.si = si


class _Err:
    __slots__ = ("si", "exc")

    def __init__(self, si: int, exc: BaseException):
        self.si = si
        self.exc = exc


def is_live_source(src: Any) -> bool:
    """Whether reading ``src`` may block the reader for an unbounded time (sockets, thread-backed
    push sources, paced generators, rank-0-read replicated streams). Sources say so themselves
    with a ``live`` attribute; push-only ``SourceFunction``s are live by construction."""
    from .functions import SourceFunction
    from .sources import ReplicatedSource, ThreadedSource

    flag = getattr(src, "live", None)
    if flag is not None:
        return bool(flag() if callable(flag) else flag)
    if isinstance(src, (ThreadedSource, ReplicatedSource)):
        return True
    if isinstance(src, SourceFunction) and type(src).iterate is SourceFunction.iterate:
        return True
    if callable(getattr(src, "run", None)) and not hasattr(src, "__iter__") and \
            not callable(getattr(src, "iterate", None)):
        return True
    return False


class DeterministicInputs:
    """Reproducible merge of pull sources (see module docstring)."""

    def __init__(self, sources: List[Any], readers: dict, chunk: int = 1024):
        self.sources = sources
        self.readers = readers
        self.chunk = int(chunk)

    def __iter__(self) -> Iterator[Any]:
        sources = self.sources
        iters = [(n, iter(self.readers[id(n)])) for n in sources]
        if len(sources) == 1 and self.chunk > 1 and is_chunkable_source(sources[0].source):
            n, it = iters[0]
            size = self.chunk
            direct = self.readers[id(n)].chunks(size)
            if direct is not None:
                for pairs in direct:
                    yield Chunk(n, pairs)
                return
            while True:
                pairs = list(itertools.islice(it, size))
                if not pairs:
                    return
                yield Chunk(n, pairs) if len(pairs) > 1 else (n, pairs[0][0], pairs[0][1])
        timed = len(sources) > 1 and all(n.timestamp_fn is not None for n in sources)
        if timed:
            heap = []
            for si, (n, it) in enumerate(iters):
                for g, v in it:
                    heapq.heappush(heap, (n.timestamp_fn(v), si, next(_seq), n, g, v))
                    break
            while heap:
                _, si, _, n, g, v = heapq.heappop(heap)
                yield n, g, v
                for ng, nv in iters[si][1]:
                    heapq.heappush(heap, (n.timestamp_fn(nv), si, next(_seq), n, ng, nv))
                    break
            return
        live = list(iters)
        while live:
            nxt = []
            for n, it in live:
                try:
                    g, v = next(it)
                except StopIteration:
                    continue
                yield n, g, v
                nxt.append((n, it))
            live = nxt

    def close(self) -> None:
        pass


class LiveInputs:
    """Available-first multiplexer over reader threads (see module docstring).

    ``capacity`` bounds the chunks queued per source. Non-live sources (collections, columnar
    batches) hand over chunks of up to ``chunk`` elements per queue operation; live sources hand
    over every element as soon as it is read (a chunk could otherwise hold a record back while the
    source blocks)."""

    def __init__(self, sources: List[Any], readers: dict, clock: Clock, capacity: int = 64, chunk: int = 256,
                 poll_s: float = 0.05):
        self.sources = sources
        self.readers = readers
        self.clock = clock
        self.poll_s = float(poll_s)
        self.q: "queue.Queue" = queue.Queue()
        self._sems = [threading.Semaphore(max(1, int(capacity))) for _ in sources]
        self._chunk = [1 if is_live_source(n.source) else max(1, int(chunk)) for n in sources]
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._active = len(sources)
        self._started = False

    # ------------------------------------------------------------------ reader threads
    def start(self) -> "LiveInputs":
        if self._started:
            return self
        self._started = True
        for si, n in enumerate(self.sources):
            t = threading.Thread(target=self._pump, args=(si, n), name=f"source-reader-{n.name}-{si}", daemon=True)
            self._threads.append(t)
            t.start()
        return self

    def _put_chunk(self, si: int, chunk: list) -> bool:
        sem = self._sems[si]
        while not sem.acquire(timeout=0.1):
            if self._stop.is_set():
                return False
        if self._stop.is_set():
            return False
        self.q.put((si, chunk))
        return True

    def _pump(self, si: int, node: Any) -> None:
        set_current_clock(self.clock)  # sources sleeping on the job clock just sleep (not the owner thread)
        reader = self.readers[id(node)]
        size = self._chunk[si]
        try:
            buf: list = []
            for g, v in reader:
                if self._stop.is_set():
                    return
                buf.append((g, v))
                if len(buf) >= size:
                    if not self._put_chunk(si, buf):
                        return
                    buf = []
            if buf and not self._put_chunk(si, buf):
                return
        except BaseException as e:  # noqa: BLE001 - re-raised on the job thread
            self.q.put(_Err(si, e))
        finally:
            self.q.put(_Eos(si))

    # ------------------------------------------------------------------ control items
    def inject(self, marker: Marker) -> None:
        """Thread-safe: ``marker`` is processed after every element enqueued before it."""
        self.q.put(marker)

    # ------------------------------------------------------------------ job thread
    def _get(self):
        try:
            return self.clock.get(self.q, timeout=self.poll_s)
        except queue.Empty:
            return IDLE

    def __iter__(self) -> Iterator[Any]:
        self.start()
        nodes = self.sources
        while self._active > 0:
            item = self._get()
            if type(item) is tuple:
                si, chunk = item
                self._sems[si].release()
                if len(chunk) > 1:
                    yield Chunk(nodes[si], chunk)
                else:
                    g, v = chunk[0]
                    yield nodes[si], g, v
            elif isinstance(item, _Eos):
                self._active -= 1
            elif isinstance(item, _Err):
                raise item.exc
            else:
                yield item

    def markers(self) -> Iterator[Marker]:
        """After end of input: barriers / stop / idle wake-ups still arriving (a distributed job
        takes the checkpoints its peers trigger until every rank has finished)."""
        while True:
            item = self._get()
            if isinstance(item, Marker):
                yield item
            elif isinstance(item, _Err):
                raise item.exc
            elif type(item) is tuple:  # pragma: no cover - sources are exhausted
                METRICS.inc("inputs.late_elements")

    def close(self) -> None:
        self._stop.set()
        for n in self.sources:
            cancel = getattr(n.source, "cancel", None)
            if callable(cancel):
                try:
                    cancel()
                except Exception:  # noqa: BLE001
                    pass


__all__ = ["Chunk", "DeterministicInputs", "IDLE", "LiveInputs", "Marker", "is_chunkable_source",
           "is_live_source"]
