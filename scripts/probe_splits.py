#!/usr/bin/env python3
"""Kernel-only time of small batches of the headline GBDT vs the tree-split count (tree-parallel
workgroups + reduce), to pick the latency path's split policy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=1000, depth=6, n_features=32))
    plan = c.plan("cuda:0")
    for n in (256, 1024, 4096, 16384, 65536):
        X = torch.from_numpy(stream_matrix(n, 32, seed=3)).cuda()
        s, v = plan.alloc_outputs(n)
        res = {"rows": n, "auto": plan._auto_splits(n)}
        for sp in (1, 4, 8, 16, 32, 62, 125, 250):
            for _ in range(3):
                plan.launch(X, s, v, splits=sp)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                plan.launch(X, s, v, splits=sp)
            e1.record()
            torch.cuda.synchronize()
            res[f"s{sp}_us"] = round(e0.elapsed_time(e1) / 50 * 1e3, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
