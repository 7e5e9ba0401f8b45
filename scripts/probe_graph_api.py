#!/usr/bin/env python3
"""Public small-batch latency (``model.predict(RecordBatch).wait()``) of multi-kernel plans with
and without HIP-graph replay (``ScoringConfig.graph_max_rows``)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from flink_jpmml_amd import PmmlModel
    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.bench.synth import mlp_pmml, segmented_pmml, stream_matrix
    from flink_jpmml_amd.config import ScoringConfig

    models = {"wide_mlp": (mlp_pmml(n_features=32, hidden=(1024, 1024, 512)), "bf16"),
              "segmented_median": (segmented_pmml("median", False, n_segments=5, seed=7), "fp32")}
    for name, (txt, prec) in models.items():
        for gmr in (0, 16384):
            m = PmmlModel.from_string(txt).bind(device="cuda:0", config=ScoringConfig(
                device="cuda:0", precision=prec, graph_max_rows=gmr, fallback="error"))
            for n in (256, 4096):
                rb = RecordBatch(torch.from_numpy(stream_matrix(n, m.evaluator.model.n_features, seed=2)).pin_memory())
                for _ in range(20):
                    m.predict(rb).wait()
                lat = []
                for _ in range(200):
                    t0 = time.perf_counter()
                    m.predict(rb).wait()
                    lat.append((time.perf_counter() - t0) * 1e6)
                print(json.dumps({"model": name, "plan": type(m.scorer.plan).__name__, "graph_max_rows": gmr,
                                  "rows": n, "p50_us": float(np.percentile(lat, 50)),
                                  "p99_us": float(np.percentile(lat, 99)),
                                  "replays": getattr(getattr(m.scorer, "_graphs", None), "replays", 0)}), flush=True)


if __name__ == "__main__":
    main()
