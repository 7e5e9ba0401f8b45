#!/usr/bin/env python3
"""Wide-layer GEMM ceiling check: the fused wide-MLP plan (ops/csrc/gemm.hip) against hipBLASLt
(torch.matmul) on the same layer shapes, 1M device-resident rows, bf16 and fp32. Prints one JSON
line per (hidden, precision): kernel-only ms and TFLOP/s of both, and the per-layer BLAS times."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5, rounds=5):
    import numpy as np
    import torch

    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return float(np.median(ts))


def main():
    import torch

    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rows = int(os.environ.get("ROWS", 1 << 20))
    for hidden in [(1024, 1024, 1024), (1024, 1024, 512), (2048, 2048)]:
        for prec in ("bf16", "fp32"):
            c = CompiledPmml.from_string(mlp_pmml(n_features=32, hidden=hidden, seed=4))
            plan = c.plan("cuda:0", precision=prec, mlp_impl="wide")
            X = torch.from_numpy(stream_matrix(rows, 32, seed=1)).cuda()
            s, v = plan.alloc_outputs(rows)
            dims = (32,) + hidden + (1,)
            flops = 2.0 * rows * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
            ms = timeit(lambda: plan.launch(X, s, v))
            dt = torch.bfloat16 if prec == "bf16" else torch.float32
            layers = []
            blas_total = 0.0
            for k, m in zip(dims[:-1], dims[1:]):
                A = torch.randn(rows, max(k, 64), device="cuda", dtype=dt)
                W = torch.randn(max(k, 64), m, device="cuda", dtype=dt)
                t = timeit(lambda: torch.matmul(A, W))
                layers.append({"K": k, "M": m, "blas_ms": t, "blas_tflops": 2.0 * rows * k * m / t / 1e9})
                blas_total += t
            print(json.dumps({"hidden": hidden, "precision": prec, "plan_ms": ms, "plan_tflops": flops / ms / 1e9,
                              "blas_gemm_only_ms": blas_total, "blas_tflops": flops / blas_total / 1e9,
                              "layers": layers}), flush=True)


if __name__ == "__main__":
    main()
