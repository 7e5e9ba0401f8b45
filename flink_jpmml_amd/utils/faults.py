"""Deterministic fault injection and rank-failure detection.

The reference has no fault injection: its recovery story is "kill a TaskManager by hand while
`CheckpointEvaluate` runs" (`flink-jpmml-examples/README.md:28-68`) and Flink's restart
strategy. Here failures are injectable from tests and from the environment so every recovery
path is exercised deterministically:

* ``fail_load`` — reading a model whose path contains the pattern raises ``OSError`` (the
  operators turn it into the reference's fatal :class:`ModelLoadingException`);
* ``corrupt_pmml`` — the document read for a matching path is truncated (a torn / partial file:
  the parser must fail loudly, never score with half a model);
* ``tear_pmml`` — a span of bytes is deleted from the middle of a matching document, at a node
  boundary (``…"/>\n <Node id="7" …`` loses ``"/>\n <Node id=``): a torn write inside a large
  ensemble, which the streaming tree scanner must refuse like the DOM parser does;
* ``kill_rank`` — rank ``r`` dies (``os._exit``) when it reaches micro-batch ``n`` of the
  distributed serving loop; the survivors' next collective fails or times out and
  :class:`Watchdog` / :func:`guarded_collective` turn that into a :class:`RankFailure` so the job
  restarts from the last checkpoint manifest (`stream/state.py`).

Environment form (read once by :func:`injector`): ``FJA_FAULTS="fail_load=bad.xml;
corrupt_pmml=torn;tear_pmml=gbdt;kill_rank=1@3"`` (``;``-separated, ``kill_rank=<rank>@<batch>``).
``FJA_FAULT_ATTEMPTS=k`` limits the faults to the first ``k`` attempts of a job run under the
restart supervisor (``FJA_ATTEMPT``, :mod:`flink_jpmml_amd.launch`): the restarted job runs clean.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

logger = logging.getLogger(__name__)

EXIT_KILLED_RANK = 43  # exit status of a rank killed by the injector


class RankFailure(RuntimeError):
    """A peer rank died or stopped responding (collective error or watchdog timeout)."""


@dataclass
class FaultInjector:
    fail_load: List[str] = field(default_factory=list)
    corrupt_pmml: List[str] = field(default_factory=list)
    tear_pmml: List[str] = field(default_factory=list)
    kill_rank: Dict[int, int] = field(default_factory=dict)  # rank -> micro-batch index

    @staticmethod
    def parse(spec: str) -> "FaultInjector":
        fi = FaultInjector()
        for item in filter(None, (s.strip() for s in spec.split(";"))):
            key, _, val = item.partition("=")
            if key == "fail_load":
                fi.fail_load.append(val)
            elif key == "corrupt_pmml":
                fi.corrupt_pmml.append(val)
            elif key == "tear_pmml":
                fi.tear_pmml.append(val)
            elif key == "kill_rank":
                r, _, n = val.partition("@")
                fi.kill_rank[int(r)] = int(n or 0)
            else:
                raise ValueError(f"unknown fault {key!r} in {spec!r}")
        return fi

    @property
    def active(self) -> bool:
        return bool(self.fail_load or self.corrupt_pmml or self.tear_pmml or self.kill_rank)

    # -- hooks
    def on_read(self, path: str, data: bytes) -> bytes:
        """Called by :class:`~flink_jpmml_amd.api.reader.FsReader` after the bytes are read."""
        if any(p in path for p in self.fail_load):
            raise OSError(f"injected load failure for {path}")
        if any(p in path for p in self.corrupt_pmml):
            logger.warning("fault injection: truncating %s", path)
            return data[: max(1, len(data) // 2)]
        if any(p in path for p in self.tear_pmml):
            return tear(data)
        return data

    def on_batch(self, rank: int, index: int) -> None:
        """Called by the serving loop before micro-batch ``index``; kills the configured rank."""
        n = self.kill_rank.get(rank)
        if n is not None and index >= n:
            logger.error("fault injection: killing rank %d at micro-batch %d", rank, index)
            logging.shutdown()
            os._exit(EXIT_KILLED_RANK)


def tear(data: bytes, at: Optional[int] = None, span: int = 15) -> bytes:
    """``data`` with ``span`` bytes deleted just before the first ``<Node`` at or after ``at``
    (default: the middle), so the tear splices the end of one node into the next."""
    mid = len(data) // 2 if at is None else at
    p = data.find(b"<Node", mid)
    p = mid if p < 0 else p
    lo = max(0, p - 3)
    logger.warning("fault injection: tearing %d bytes at offset %d", span, lo)
    return data[:lo] + data[lo + span:]


_INJECTOR: Optional[FaultInjector] = None


def injector() -> FaultInjector:
    """Process-wide injector (from ``FJA_FAULTS`` on first use)."""
    global _INJECTOR
    if _INJECTOR is None:
        spec = os.environ.get("FJA_FAULTS", "")
        limit = os.environ.get("FJA_FAULT_ATTEMPTS")
        if limit is not None and int(os.environ.get("FJA_ATTEMPT", "0")) >= int(limit):
            spec = ""
        _INJECTOR = FaultInjector.parse(spec)
    return _INJECTOR


def set_injector(fi: Optional[FaultInjector]) -> None:
    """Install (or with ``None`` reset to the environment's) injector — tests use this."""
    global _INJECTOR
    _INJECTOR = fi


class Watchdog:
    """Heartbeat timer: if :meth:`kick` is not called within ``timeout_s`` the ``on_timeout``
    callback runs once on the watchdog thread (default: log and abort the process with status
    :data:`EXIT_KILLED_RANK` + 1, so a supervisor restarts the job from the last manifest — a
    rank blocked inside an RCCL collective cannot be unblocked from Python)."""

    def __init__(self, timeout_s: float, on_timeout: Optional[Callable[[], None]] = None, name: str = "rank"):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout or self._abort
        self.name = name
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.fired = False
        self._t = threading.Thread(target=self._run, name=f"watchdog-{name}", daemon=True)

    def _abort(self) -> None:  # pragma: no cover - exercised through subprocess tests only
        logger.critical("watchdog %s: no progress for %.1f s, aborting", self.name, self.timeout_s)
        logging.shutdown()
        os._exit(EXIT_KILLED_RANK + 1)

    def start(self) -> "Watchdog":
        self._last = time.monotonic()
        self._t.start()
        return self

    def kick(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=5)

    def _run(self) -> None:
        period = min(0.05, self.timeout_s / 4)
        while not self._stop.wait(period):
            if time.monotonic() - self._last > self.timeout_s:
                self.fired = True
                self.on_timeout()
                return

    def __enter__(self) -> "Watchdog":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()


def guarded_collective(fn: Callable, *args, what: str = "collective", **kw):
    """Run a collective; a peer failure (connection reset, timeout, RCCL/gloo error) becomes
    :class:`RankFailure` with the original error as its cause."""
    try:
        return fn(*args, **kw)
    except RankFailure:
        raise
    except (RuntimeError, ConnectionError, TimeoutError) as e:
        raise RankFailure(f"{what} failed: a peer rank is gone or stalled ({e})") from e
