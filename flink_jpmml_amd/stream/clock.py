"""Processing-time clock + timer service of the stream runtime.

Flink operators flush on processing-time timers; the reference's example sources block in
``Thread.sleep(1000)`` between records (`E/sources/IrisSource.scala:52`). In this runtime every
blocking point of the job thread — a source sleeping until its next record, a source thread's
queue being empty — goes through the job's :class:`Clock`, which fires due timers while it waits.
A micro-batch with a ``max_batch_latency_ms`` bound is therefore flushed on time even when the
next record is seconds away.

* :class:`SystemClock` — wall time (``time.monotonic``), real sleeps cut at timer deadlines;
* :class:`ManualClock` — virtual time for deterministic tests: ``sleep(dt)`` advances time
  instantly, firing every timer whose deadline it crosses, in order.

Sources obtain the running job's clock with :func:`current_clock` (``SystemClock`` outside jobs).
"""

from __future__ import annotations

import heapq
import itertools
import queue
import threading
import time
from typing import Callable, List, Optional, Tuple

_seq = itertools.count()


class TimerService:
    """Min-heap of ``(deadline_s, callback)``; callbacks run on the job thread."""

    def __init__(self):
        self._heap: List[Tuple[float, int, Callable[[float], None]]] = []

    def register(self, deadline: float, callback: Callable[[float], None]) -> None:
        heapq.heappush(self._heap, (float(deadline), next(_seq), callback))

    def next_deadline(self) -> Optional[float]:
        return self._heap[0][0] if self._heap else None

    def fire(self, now: float) -> int:
        n = 0
        while self._heap and self._heap[0][0] <= now:
            _, _, cb = heapq.heappop(self._heap)
            cb(now)
            n += 1
        return n

    def clear(self) -> None:
        self._heap.clear()


class Clock:
    timers: TimerService

    def now(self) -> float:  # seconds
        raise NotImplementedError

    def sleep(self, dt: float) -> None:
        raise NotImplementedError

    def get(self, q: "queue.Queue", timeout: Optional[float] = None):
        """``q.get()`` that fires due timers while waiting (raises ``queue.Empty`` on timeout)."""
        raise NotImplementedError

    def fire_due(self) -> int:
        return self.timers.fire(self.now())

    def _owner_thread(self) -> bool:
        return getattr(self, "_thread", None) in (None, threading.get_ident())

    def bind_thread(self) -> None:
        """Only the job thread fires timers (a source thread sleeping on the clock just sleeps)."""
        self._thread = threading.get_ident()


class SystemClock(Clock):
    def __init__(self):
        self.timers = TimerService()
        self._thread = None

    def now(self) -> float:
        return time.monotonic()

    def sleep(self, dt: float) -> None:
        end = time.monotonic() + max(0.0, dt)
        if not self._owner_thread():
            time.sleep(max(0.0, dt))
            return
        while True:
            now = time.monotonic()
            self.timers.fire(now)
            if now >= end:
                return
            nd = self.timers.next_deadline()
            time.sleep(max(0.0, min(end, nd if nd is not None else end) - now))

    def get(self, q: "queue.Queue", timeout: Optional[float] = None):
        end = None if timeout is None else time.monotonic() + timeout
        while True:
            now = time.monotonic()
            if self._owner_thread():
                self.timers.fire(now)
            nd = self.timers.next_deadline() if self._owner_thread() else None
            lim = end
            if nd is not None:
                lim = nd if lim is None else min(lim, nd)
            wait = None if lim is None else max(0.0, lim - now)
            try:
                return q.get(timeout=wait) if wait is not None else q.get()
            except queue.Empty:
                if end is not None and time.monotonic() >= end:
                    raise


class ManualClock(Clock):
    """Virtual time: ``sleep(dt)`` jumps from timer deadline to timer deadline (firing each) and
    then to ``now + dt``. ``advance`` is an alias usable from tests."""

    def __init__(self, start: float = 0.0):
        self.timers = TimerService()
        self._now = float(start)
        self._thread = None

    def now(self) -> float:
        return self._now

    def sleep(self, dt: float) -> None:
        end = self._now + max(0.0, dt)
        while True:
            nd = self.timers.next_deadline()
            if nd is None or nd > end:
                break
            self._now = max(self._now, nd)
            self.timers.fire(self._now)
        self._now = end
        self.timers.fire(self._now)

    advance = sleep

    def get(self, q: "queue.Queue", timeout: Optional[float] = None):
        return q.get(timeout=timeout)


_local = threading.local()
_default = SystemClock()


def current_clock() -> Clock:
    """The clock of the job running on this thread (a process-wide SystemClock otherwise)."""
    return getattr(_local, "clock", None) or _default


def set_current_clock(clock: Optional[Clock]) -> None:
    _local.clock = clock


__all__ = ["Clock", "ManualClock", "SystemClock", "TimerService", "current_clock", "set_current_clock"]
