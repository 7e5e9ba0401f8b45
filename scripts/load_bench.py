#!/usr/bin/env python3
"""Large-model load benchmark: a scikit-learn-style random forest of the size
the reference advertises ("several hundreds of MegaBytes", `README.md:239-242`) — by default 300
trees, depth <= 14, 32 features, 3 classes (~206 MB of PMML) — loaded through the operators' path
(read bytes -> streaming tree scanner -> flat arrays -> evaluator -> lowering -> device plan).

    python scripts/load_bench.py [--trees 300 --depth 14] [--device cuda]

Prints one JSON line: document size, load seconds (with the phase split), peak RSS growth."""

from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rss_mb() -> float:
    with open("/proc/self/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return float("nan")


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--trees", type=int, default=300)
    p.add_argument("--depth", type=int, default=14)
    p.add_argument("--features", type=int, default=32)
    p.add_argument("--p-split", type=float, default=0.85)
    p.add_argument("--device", default=None)
    p.add_argument("--path", default=None, help="existing PMML file (skip generation)")
    a = p.parse_args(argv)
    path = a.path
    if path is None:
        from flink_jpmml_amd.bench.synth import random_forest_pmml

        path = os.path.join(tempfile.gettempdir(), f"rf_{a.trees}_{a.depth}_{a.features}.pmml")
        if not os.path.exists(path):
            with open(path, "w") as fh:
                fh.write(random_forest_pmml(n_trees=a.trees, depth=a.depth, n_features=a.features, n_classes=3,
                                            seed=1, p_split=a.p_split))
    import torch  # noqa: F401 - imported before the timed region (a cold torch import is seconds)

    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.runtime.loading import load_local
    from flink_jpmml_amd.utils.metrics import METRICS

    device = a.device
    if device is not None:
        torch.zeros(1, device=device)  # HIP context up front
    base_rss = rss_mb()
    t0 = time.perf_counter()
    lm = load_local(path, device, ScoringConfig(device=device, fallback="error") if device else None)
    if device is not None:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    plan = getattr(lm.model.scorer, "plan", None)
    print(json.dumps({
        "metric": "large PMML load", "path": path, "bytes": os.path.getsize(path), "trees": a.trees,
        "depth": a.depth, "device": device, "load_s": dt, "rss_before_mb": base_rss, "rss_after_mb": rss_mb(),
        "peak_rss_mb": peak, "materialized_nodes": METRICS.counters.get("pmml.flat_materialized_nodes", 0),
        "layout": getattr(plan, "layout", None), "head_depth": getattr(plan, "head_depth", None),
        "chunk_trees": getattr(plan, "chunk_trees", None), "sha256": lm.sha256[:16]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
