#!/usr/bin/env python3
"""Per-record stream throughput: the reference's call pattern (one FlinkML-style ``DenseVector``
per element, ``quickEvaluate`` → ``(Prediction, vector)`` per element, `S/package.scala:138-142`)
through the DSL with micro-batching (``batch_size``), on the host oracle or the GPU.

    python scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt
    python scripts/per_record_bench.py --device cuda --api to_batches   # columnar adapter

Prints one JSON line (records/s of the timed ``env.execute``; vectors are built beforehand, like
any in-memory source)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--device", default=None)
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--batch-size", type=int, default=65536)
    p.add_argument("--model", choices=["kmeans", "gbdt"], default="kmeans")
    p.add_argument("--api", choices=["quick", "evaluate", "to_batches"], default="quick")
    p.add_argument("--repeats", type=int, default=3)
    a = p.parse_args(argv)
    import numpy as np

    from flink_jpmml_amd import DenseVector, ModelReader
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.stream import CollectSink, StreamExecutionEnvironment

    d = tempfile.mkdtemp()
    if a.model == "kmeans":
        from flink_jpmml_amd.assets import write_fixtures

        path, F = write_fixtures(d)["kmeans"], 4
    else:
        from flink_jpmml_amd.bench.synth import gbdt_pmml

        F = 32
        path = os.path.join(d, "gbdt.pmml")
        with open(path, "w") as fh:
            fh.write(gbdt_pmml(n_trees=1000, depth=6, n_features=F, seed=0))
    X = np.random.default_rng(0).uniform(0.2, 7.0, size=(a.rows, F))
    vecs = [DenseVector(r) for r in X]
    cfg = ScoringConfig(device=a.device, batch_size=a.batch_size, fallback="error" if a.device else "warn")
    best = None
    for _ in range(a.repeats):
        env = StreamExecutionEnvironment(config=cfg)
        src = env.from_collection(vecs)
        sink = CollectSink()
        if a.api == "quick":
            src.quick_evaluate(ModelReader(path)).add_sink(sink)
        elif a.api == "evaluate":
            src.evaluate(ModelReader(path), lambda v, m: (v, m.predict(v))).add_sink(sink)
        else:
            src.to_batches(lambda v: v.data, batch_rows=a.batch_size).quick_evaluate(ModelReader(path)) \
               .unbatch().add_sink(sink)
        t0 = time.perf_counter()
        env.execute("per-record")
        dt = time.perf_counter() - t0
        assert len(sink.values) == a.rows, len(sink.values)
        best = dt if best is None else min(best, dt)
    print(json.dumps({"metric": "per-record quick_evaluate records/s", "api": a.api, "model": a.model,
                      "device": a.device, "rows": a.rows, "batch_size": a.batch_size,
                      "records_per_s": a.rows / best, "seconds": best}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
