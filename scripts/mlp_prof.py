#!/usr/bin/env python3
"""Wide MLP kernel-only run for rocprofv3 (per-kernel times of the layer GEMMs): HIDDEN layers
(default 1024,1024,1024), N_FEATURES inputs (32), 1M device-resident rows, PREC precision, ITERS launches."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rows = int(os.environ.get("ROWS", 1 << 20))
    hidden = tuple(int(h) for h in os.environ.get("HIDDEN", "1024,1024,1024").split(","))
    prec = os.environ.get("PREC", "bf16")
    iters = int(os.environ.get("ITERS", 10))
    nf = int(os.environ.get("N_FEATURES", 32))
    c = CompiledPmml.from_string(mlp_pmml(n_features=nf, hidden=hidden, seed=4))
    plan = c.plan("cuda:0", precision=prec, mlp_impl="wide")
    plan.fuse_input = os.environ.get("FUSE_INPUT", "1") == "1"
    plan.fuse_head = os.environ.get("FUSE_HEAD", "1") == "1"
    plan.gemm_flags = int(os.environ.get("GEMM_FLAGS", "0"), 0)
    X = torch.from_numpy(stream_matrix(rows, nf, seed=1)).cuda()
    s, v = plan.alloc_outputs(rows)
    plan.launch(X, s, v)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        plan.launch(X, s, v)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    print(json.dumps({"hidden": hidden, "precision": prec, "rows": rows, "ms": ms, "plan": type(plan).__name__,
                      "fuse_input": plan.fuse_input, "fuse_head": plan.fuse_head, "gemm_flags": plan.gemm_flags}))


if __name__ == "__main__":
    main()
