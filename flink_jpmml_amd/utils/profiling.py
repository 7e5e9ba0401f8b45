"""Profiler ranges around the scoring pipeline stages (ingest / H2D / kernel / D2H / gather).

Uses ``torch.profiler.record_function`` (which also emits roctx ranges visible to rocprofv3's
marker tracing) when torch is importable; a no-op otherwise. Enable with ``FJA_PROFILE=1``.
``FJA_PROFILE=2`` instead accumulates each range's host wall time into the metrics counters
``prange_us.<name>`` (microseconds) and ``prange_n.<name>`` (entries) — a cheap per-stage
breakdown of the job thread that ``bench.py`` prints with its other counters.
"""

from __future__ import annotations

import os
import time
from contextlib import contextmanager, nullcontext

ENABLED = os.environ.get("FJA_PROFILE", "0") == "1"
TIMING = os.environ.get("FJA_PROFILE", "0") == "2"


@contextmanager
def prange(name: str):
    if TIMING:
        from .metrics import METRICS

        t0 = time.perf_counter()
        try:
            yield
        finally:
            METRICS.inc(f"prange_us.{name}", int((time.perf_counter() - t0) * 1e6))
            METRICS.inc(f"prange_n.{name}")
        return
    if not ENABLED:
        yield
        return
    try:
        from torch.profiler import record_function
    except ImportError:  # pragma: no cover
        with nullcontext():
            yield
        return
    with record_function(name):
        yield
