"""Probe: where does the back-to-back pipelined step lose time? (variants in one process)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.engine import StreamingScorer


class NoopPlan:
    def __init__(self, p):
        self.device, self.n_features = p.device, p.n_features

    def launch(self, X, s, v, stream=None):
        pass


def run(sc, Xh, sh, vh, steps=10):
    for _ in range(2):
        sc.wait(sc.submit(Xh, sh, vh))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        h = sc.submit(Xh, sh, vh)
    sc.wait(h)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


c = CompiledPmml.from_string(gbdt_pmml(n_trees=1000, depth=6, n_features=32))
plan = c.plan("cuda:0")
R = 1 << 20
Xh = torch.from_numpy(stream_matrix(R, 32)).pin_memory()
sh = torch.empty(R).pin_memory()
vh = torch.empty(R, dtype=torch.uint8).pin_memory()
res = {}
for mb in (131072, 262144, 65536):
    for depth in (3, 4):
        res[f"direct_mb{mb}_d{depth}"] = run(StreamingScorer(plan, mb, depth, R), Xh, sh, vh)
        res[f"copy_mb{mb}_d{depth}"] = run(StreamingScorer(plan, mb, depth, R, direct_host_output=False), Xh, sh, vh)
res["direct_nomirror_mb131072"] = run(StreamingScorer(plan, 131072, 4, R, keep_device_output=False), Xh, sh, vh)
res["no_d2h"] = run(StreamingScorer(plan, 131072, 4, R), Xh, None, None)
res["h2d_only"] = run(StreamingScorer(NoopPlan(plan), 131072, 4, R), Xh, None, None)
res["h2d_d2h_only"] = run(StreamingScorer(NoopPlan(plan), 131072, 4, R, direct_host_output=False), Xh, sh, vh)
Xd = Xh.cuda()
s = torch.empty(R, device="cuda")
v = torch.empty(R, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    for i in range(0, R, 131072):
        plan.launch(Xd[i:i + 131072], s[i:i + 131072], v[i:i + 131072])
torch.cuda.synchronize()
res["kernels_only_mb131072"] = (time.perf_counter() - t0) / 10 * 1e3
print(json.dumps(res))
