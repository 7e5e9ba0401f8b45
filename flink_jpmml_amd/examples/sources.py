"""Example sources (reference `E/sources/*.scala`, `E/model/Iris.scala`, `E/model/Utils.scala`).

* :class:`IrisSource` — Iris-like events (4 uniform features in [0.2, 6.0], one decimal), tagged
  with a random model id from ``ids``. The reference emits 1 record/s via ``Thread.sleep(1000)``
  and crashes with an empty id list (`E/sources/IrisSource.scala:39,45`); here the rate is a
  parameter (``rate=None`` = as fast as possible) and no ids give untagged events.
* :class:`ControlSource` — ``AddMessage``s for ``(uuid, path)`` pairs under the ``loop`` /
  ``random`` (infinite) or ``finite`` policies (`E/sources/ControlSource.scala:48-57`).
"""

from __future__ import annotations

import random
import time
import uuid
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

from ..api.vectors import DenseVector
from ..domain.control import AddMessage
from ..stream.clock import current_clock
from ..stream.functions import SourceContext, SourceFunction


def now_ms() -> int:
    return int(time.time() * 1000)


@dataclass(frozen=True)
class Iris:
    """``case class Iris(modelId, 4 doubles, occurredOn) extends BaseEvent`` (`E/model/Iris.scala:25-33`)."""

    model_id: Optional[str]
    sepal_length: float
    sepal_width: float
    petal_length: float
    petal_width: float
    occurred_on: int

    def to_vector(self) -> DenseVector:
        return DenseVector(self.sepal_length, self.sepal_width, self.petal_length, self.petal_width)

    toVector = to_vector  # noqa: N815


def ids_and_paths(paths: Sequence[str]) -> Dict[str, str]:
    """Random UUID per model path (`E/model/Utils.scala:26-37`)."""
    return {str(uuid.uuid4()): p for p in paths}


class IrisSource(SourceFunction):
    def __init__(self, ids: Optional[Sequence[str]] = None, n: Optional[int] = 100, rate: Optional[float] = None,
                 seed: int = 0, version: int = 1):
        self.ids = list(ids or [])
        self.n = n
        self.rate = rate
        self.seed = seed
        self.version = version
        self._running = True

    @property
    def live(self) -> bool:
        """Paced sources block between records: the runtime reads them on a thread of their own."""
        return bool(self.rate)

    def _gen(self) -> Iterator[Iris]:
        rng = random.Random(self.seed)
        i = 0
        while self._running and (self.n is None or i < self.n):
            vals = [round(rng.uniform(0.2, 6.0), 1) for _ in range(4)]
            mid = f"{rng.choice(self.ids)}_{self.version}" if self.ids else None
            yield Iris(mid, *vals, now_ms())
            i += 1
            if self.rate:
                current_clock().sleep(1.0 / self.rate)  # the job clock fires due timers meanwhile

    def run(self, ctx: SourceContext) -> None:
        for ev in self._gen():
            ctx.collect(ev)

    def iterate(self):
        return self._gen()

    def cancel(self) -> None:
        self._running = False


class ControlSource(SourceFunction):
    """Control stream generator. ``policy``: ``finite`` (one Add per model), ``loop`` (cycle through
    the models forever / ``n`` messages), ``random`` (random model each time)."""

    POLICIES = ("finite", "loop", "random")

    def __init__(self, ids_paths: Dict[str, str], policy: str = "finite", n: Optional[int] = None,
                 max_interval_ms: int = 0, seed: int = 0, version: int = 1):
        if policy not in self.POLICIES:
            raise ValueError(f"gen-policy must be one of {self.POLICIES}")
        self.items: List[Tuple[str, str]] = list(ids_paths.items())
        self.policy = policy
        self.n = n
        self.max_interval_ms = max_interval_ms
        self.seed = seed
        self.version = version
        self._running = True

    @property
    def live(self) -> bool:
        return bool(self.max_interval_ms)

    def _gen(self) -> Iterator[AddMessage]:
        rng = random.Random(self.seed)
        count = 0
        if self.policy == "finite":
            seq = iter(self.items)
        elif self.policy == "loop":
            seq = (self.items[i % len(self.items)] for i in range(10 ** 12))
        else:
            seq = (rng.choice(self.items) for _ in range(10 ** 12))
        for mid, path in seq:
            if not self._running or (self.n is not None and count >= self.n):
                break
            if self.max_interval_ms:
                current_clock().sleep(rng.uniform(0, self.max_interval_ms) / 1000.0)
            yield AddMessage(mid, self.version, path, now_ms())
            count += 1

    def run(self, ctx: SourceContext) -> None:
        for m in self._gen():
            ctx.collect(m)

    def iterate(self):
        return self._gen()

    def cancel(self) -> None:
        self._running = False
