#!/usr/bin/env python3
"""cProfile of the public small-batch path ``model.predict(RecordBatch).wait()`` (host overhead
around the ~60 us of GPU work), top functions by own time."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from flink_jpmml_amd import PmmlModel
    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.config import ScoringConfig

    txt = gbdt_pmml(n_trees=1000, depth=6, n_features=32)
    model = PmmlModel.from_string(txt).bind(device="cuda:0", config=ScoringConfig(device="cuda:0"))
    rb = RecordBatch(torch.from_numpy(stream_matrix(int(os.environ.get("ROWS", "4096")), 32, seed=3)).pin_memory())
    for _ in range(50):
        model.predict(rb).wait()
    n = 2000
    lat = []
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        t0 = time.perf_counter()
        model.predict(rb).wait()
        lat.append(time.perf_counter() - t0)
    pr.disable()
    print(f"p50 under cProfile: {np.percentile(lat, 50) * 1e6:.1f} us")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
