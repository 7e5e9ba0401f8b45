"""Default vs full sweep of the randomized GPU suites.

The round-end GPU run (``pytest -m gpu``) has a fixed time budget, so every randomized GPU file
runs a representative slice of its seeds by default; ``FJA_FULL_SUITE=1`` runs every seed (the
builder's full sweep through ``gpurun``, log committed under ``profiles/``). CPU-side twins of the
same fuzzers always run their full seed ranges."""

import os

FULL = os.environ.get("FJA_FULL_SUITE") == "1"


def gpu_seeds(full: int, quick: int):
    """``range(full)`` under ``FJA_FULL_SUITE=1``, else the first ``quick`` seeds plus a spread
    of later ones (so the slice still reaches the generators' late branches)."""
    if FULL or quick >= full:
        return list(range(full))
    head = list(range(max(1, quick // 2)))
    rest = quick - len(head)
    step = max(1, (full - len(head)) // max(1, rest))
    tail = list(range(len(head), full, step))[:rest]
    return head + tail
