"""Host-path throughput of the 1000-tree GBDT (native walker): batch oracle and per-record predict."""
import json
import sys
import time

sys.path.insert(0, ".")
from flink_jpmml_amd import DenseVector  # noqa: E402
from flink_jpmml_amd.api.pmml_model import PmmlModel  # noqa: E402
from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.runtime.compiled import CompiledPmml  # noqa: E402

doc = gbdt_pmml(n_trees=1000, depth=6, n_features=32, seed=0)
c = CompiledPmml.from_string(doc)
X = stream_matrix(65536, 32, seed=1, missing_rate=0.02).astype("float64")
c.score_matrix_oracle(X[:64])
t = time.perf_counter()
c.score_matrix_oracle(X)
batch = len(X) / (time.perf_counter() - t)
m = PmmlModel.from_string(doc)
m.predict_batch(X[:64])
t = time.perf_counter()
m.predict_batch(X)
pbatch = len(X) / (time.perf_counter() - t)
vecs = [DenseVector(r) for r in X[:300]]
m.predict(vecs[0])
t = time.perf_counter()
for v in vecs:
    m.predict(v)
rec = len(vecs) / (time.perf_counter() - t)
from flink_jpmml_amd.bench.synth import random_forest_pmml  # noqa: E402

rf = CompiledPmml.from_string(random_forest_pmml(n_trees=500, depth=8, n_features=32, n_classes=3, seed=0))
rf.score_matrix_oracle(X[:64])
t = time.perf_counter()
rf.score_matrix_oracle(X)
rf_batch = len(X) / (time.perf_counter() - t)
print(json.dumps({"host_batch_records_per_s": batch, "host_per_record_predict_per_s": rec, "host_predict_batch_per_s": pbatch, "trees": 1000, "depth": 6,
                  "rf500x8_host_batch_records_per_s": rf_batch}))
