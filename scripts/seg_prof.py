#!/usr/bin/env python3
"""Segmented MiningModel, one 1M-row device batch per launch, for rocprofv3 --kernel-trace: the
kernels a segmented batch costs (K tree segments -> one multi-segment walk + the fused
predicate/aggregation kernel). Prints the plan's segment layouts and the ms per batch."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rows = int(os.environ.get("ROWS", 1 << 20))
    iters = int(os.environ.get("ITERS", 5))
    out = []
    for method, cls in (("selectFirst", False), ("max", True), ("median", False)):
        c = CompiledPmml.from_string(segmented_pmml(method, cls, n_segments=8, n_classes=3, seed=3))
        plan = c.plan("cuda:0")
        X = torch.from_numpy(stream_matrix(rows, c.n_features, seed=1, missing_rate=0.02)).cuda()
        s, v = plan.alloc_outputs(rows)
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            plan.launch(X, s, v)
        torch.cuda.synchronize()
        out.append({"method": method, "classification": cls, "plan": type(plan).__name__,
                    "layouts": [getattr(p, "layout", type(p).__name__) for p in getattr(plan, "subs", [])],
                    "multi_groups": [len(g["idx"]) for g in (getattr(plan, "_multi", None) or [])],
                    "ms_per_batch": (time.perf_counter() - t0) / iters * 1e3, "rows": rows})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
