"""Where a per-record device ``predict`` spends its time (1000-tree GBDT, steady state): cProfile of
5000 calls plus the wall rate."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from flink_jpmml_amd import DenseVector  # noqa: E402
from flink_jpmml_amd.api.pmml_model import PmmlModel  # noqa: E402
from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.config import ScoringConfig  # noqa: E402

m = PmmlModel.from_string(gbdt_pmml(n_trees=1000, depth=6, n_features=32, seed=0))
m.bind("cuda:0", ScoringConfig(device="cuda:0", fallback="error"))
assert m.on_device
vecs = [DenseVector(r) for r in stream_matrix(5000, 32, seed=5, missing_rate=0.02).astype(np.float64)]
for v in vecs[:200]:
    m.predict(v)
t = time.perf_counter()
for v in vecs:
    m.predict(v)
rate = len(vecs) / (time.perf_counter() - t)
pr = cProfile.Profile()
pr.enable()
for v in vecs:
    m.predict(v)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
print(f"per-record device predict: {rate:.0f} records/s")
print(s.getvalue())
