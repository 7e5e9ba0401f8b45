"""Per-record device predict rate vs the number of tree slices of the 1-row launch (1000-tree GBDT)."""
import json
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from flink_jpmml_amd import DenseVector  # noqa: E402
from flink_jpmml_amd.api.pmml_model import PmmlModel  # noqa: E402
from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.config import ScoringConfig  # noqa: E402

doc = gbdt_pmml(n_trees=1000, depth=6, n_features=32, seed=0)
vecs = [DenseVector(r) for r in stream_matrix(3000, 32, seed=5, missing_rate=0.02).astype(np.float64)]
ref = None
for k in (16, 1, 2, 4, 8, 32, 16):
    m = PmmlModel.from_string(doc)
    m.bind("cuda:0", ScoringConfig(device="cuda:0", fallback="error"))
    m.scorer.plan.splits = k
    out = [m.predict(v).value.get_or_else(float("nan")) for v in vecs[:300]]
    t = time.perf_counter()
    for v in vecs:
        m.predict(v)
    rate = len(vecs) / (time.perf_counter() - t)
    same = ref is None or np.allclose(out, ref, rtol=0, atol=1e-5, equal_nan=True)
    ref = ref if ref is not None else out
    print(json.dumps({"splits": k, "records_per_s": round(rate), "scores_match": bool(same)}), flush=True)
