"""Probe: host-side cost of one kernel launch and of StreamingScorer.submit pieces."""
import json
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.engine import StreamingScorer

c = CompiledPmml.from_string(gbdt_pmml(n_trees=1000, depth=6, n_features=32))
plan = c.plan("cuda:0")
X = torch.from_numpy(stream_matrix(131072, 32)).cuda()
s = torch.empty(131072, device="cuda")
v = torch.empty(131072, dtype=torch.uint8, device="cuda")
res = {}
for variant in (1, 0):
    plan.variant = variant
    plan._args = {}
    if variant == 0:
        plan.chunk_trees = 9
    torch.cuda.synchronize()
    ts = []
    for i in range(10):
        t0 = time.perf_counter()
        plan.launch(X, s, v)
        ts.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    res[f"launch_us_variant{variant}"] = sorted(ts)
plan.variant = 1
plan._args = {}
plan.chunk_trees = 79
Xh = torch.from_numpy(stream_matrix(1 << 20, 32)).pin_memory()
sh = torch.empty(1 << 20).pin_memory()
vh = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
sc = StreamingScorer(plan, micro_batch=131072, depth=4, max_rows=1 << 20)
for i in range(3):
    sc.wait(sc.submit(Xh, sh, vh))
ts = []
for i in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = sc.submit(Xh, sh, vh)
    t1 = time.perf_counter()
    sc.wait(h)
    t2 = time.perf_counter()
    ts.append(((t1 - t0) * 1e3, (t2 - t0) * 1e3))
res["submit_ms(call,total)"] = ts
print(json.dumps(res))
