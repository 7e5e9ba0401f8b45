#!/usr/bin/env python3
"""Host-ingest throughput of the native C++ record parser (text -> fp32 matrix) for the bench's
32-float-feature records. Prints one JSON line (records/s, MB/s) per thread count."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.native import RecordParser  # noqa: E402
from flink_jpmml_amd.runtime.compiled import CompiledPmml  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
c = CompiledPmml.from_string(gbdt_pmml(n_trees=2, depth=2, n_features=32))
X = stream_matrix(rows, 32, seed=1, missing_rate=0.01)
text = "\n".join(",".join("" if np.isnan(v) else f"{v:.7g}" for v in r) for r in X).encode() + b"\n"
out = np.empty((rows, 32), np.float32)
res = {"rows": rows, "bytes": len(text)}
for t in (1, 4, 8, 16):
    p = RecordParser(c, c.active_fields, threads=t)
    p.parse(text, out=out)
    t0 = time.perf_counter()
    for _ in range(3):
        m, _ = p.parse(text, out=out)
    dt = (time.perf_counter() - t0) / 3
    res[f"threads{t}_records_per_s"] = rows / dt
    res[f"threads{t}_MBps"] = len(text) / dt / 1e6
res["exact"] = bool(np.array_equal(np.isnan(m), np.isnan(X)))
print(json.dumps(res))
