"""Metrics registry (the reference registers none): counters + latency histograms,
exported as JSON lines.

    from flink_jpmml_amd.utils.metrics import METRICS
    METRICS.inc("records_scored", n)
    with METRICS.timer("batch_latency_ms"):
        ...
    METRICS.dump("metrics.jsonl")
"""

from __future__ import annotations

import json
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional

import numpy as np


class Metrics:
    def __init__(self, window: int = 100_000):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = defaultdict(float)
        self.samples: Dict[str, List[float]] = defaultdict(list)
        self.window = window

    def inc(self, name: str, value: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += value

    def observe(self, name: str, value: float) -> None:
        with self._lock:
            s = self.samples[name]
            s.append(value)
            if len(s) > self.window:
                del s[: len(s) - self.window]

    @contextmanager
    def timer(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.observe(name, (time.perf_counter() - t0) * 1e3)

    def summary(self) -> dict:
        with self._lock:
            out = {"counters": dict(self.counters)}
            hist = {}
            for k, v in self.samples.items():
                if v:
                    a = np.asarray(v)
                    hist[k] = {"n": int(a.size), "p50": float(np.percentile(a, 50)), "p99": float(np.percentile(a, 99)),
                               "mean": float(a.mean()), "max": float(a.max())}
            out["histograms"] = hist
            return out

    def dump(self, path: Optional[str] = None) -> str:
        line = json.dumps({"ts": time.time(), **self.summary()})
        if path:
            with open(path, "a") as fh:
                fh.write(line + "\n")
        return line

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.samples.clear()


METRICS = Metrics()
