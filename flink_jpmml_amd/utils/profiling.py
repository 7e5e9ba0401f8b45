"""Profiler ranges around the scoring pipeline stages (ingest / H2D / kernel / D2H / gather).

Uses ``torch.profiler.record_function`` (which also emits roctx ranges visible to rocprofv3's
marker tracing) when torch is importable; a no-op otherwise. Enable with ``FJA_PROFILE=1``.
"""

from __future__ import annotations

import os
from contextlib import contextmanager, nullcontext

ENABLED = os.environ.get("FJA_PROFILE", "0") == "1"


@contextmanager
def prange(name: str):
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
