#!/usr/bin/env python3
"""Interleaved A/B of wide-layer GEMM kernel variants in ONE process: N rounds x each variant,
device time per launch over 1M device-resident rows; also checks that every variant produces the
same scores as the first. Prints one JSON line per variant.

A variant is a value of ``GemmArgs.f32``'s experiment bits, set through ``plan.gemm_flags`` (the
plan ORs it into the launch). The round-3 experiments (``profiles/r3ak/``: bit 4 = LDS swizzle,
bit 5 = 4-wave pipelined loop) were measured and folded in or removed; with no experiment bits
compiled in, run it with ``VARIANTS=0`` to time the shipped kernel."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    hidden = tuple(int(x) for x in os.environ.get("HIDDEN", "1024,1024,512").split(","))
    prec = os.environ.get("PRECISION", "bf16")
    variants = [int(v, 0) for v in os.environ.get("VARIANTS", "0").split(",")]
    rows, rounds, iters = int(os.environ.get("ROWS", 1 << 20)), int(os.environ.get("ROUNDS", 5)), 5
    c = CompiledPmml.from_string(mlp_pmml(n_features=32, hidden=hidden, seed=4))
    plan = c.plan("cuda:0", precision=prec, mlp_impl="wide")
    X = torch.from_numpy(stream_matrix(rows, 32, seed=1)).cuda()
    s, v = plan.alloc_outputs(rows)
    flops = 2.0 * rows * sum(a * b for a, b in zip((32,) + hidden, hidden + (1,)))
    times = {k: [] for k in variants}
    ref = None
    for var in variants:  # warm-up + correctness
        plan.gemm_flags = var
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        if ref is None:
            ref = s.clone()
        else:
            assert torch.equal(ref, s), f"variant {var:#x} differs: max {float((ref - s).abs().max())}"
    for _ in range(rounds):
        for var in variants:
            plan.gemm_flags = var
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                plan.launch(X, s, v)
            e1.record()
            torch.cuda.synchronize()
            times[var].append(e0.elapsed_time(e1) / iters)
    for var in variants:
        t = np.array(times[var])
        print(json.dumps({"hidden": hidden, "precision": prec, "variant": hex(var), "ms_median": float(np.median(t)),
                          "ms_min": float(t.min()), "tflops_median": flops / np.median(t) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
