"""Library GEMM probe for the wide-NN layer shape (BASELINE config 4 follow-up): 1M rows x 1024 x 1024
bf16, hipBLASLt through torch (plain, bias, fused bias + ReLU epilogue) vs the repo's fused MFMA
layer kernel timings in profiles/r5q (2.14 ms storing layer). Prints one JSON line per variant."""
import json

import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


M, N, K = 1 << 20, 1024, 1024
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
wt = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)  # nn.Linear layout [out, in]
w = wt.t().contiguous()
b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
variants = {
    "mm": lambda: torch.mm(x, w, out=out),
    "addmm_bias": lambda: torch.addmm(b, x, w, out=out),
    "linear_bias": lambda: torch.nn.functional.linear(x, wt, b),
    "addmm_relu_fused": lambda: torch._addmm_activation(b, x, w),
    "addmm_then_relu": lambda: torch.relu_(torch.addmm(b, x, w, out=out)),
}
flops = 2.0 * M * N * K
for name, fn in variants.items():
    try:
        ms = bench(fn)
        print(json.dumps({"variant": name, "ms": ms, "tflops": flops / ms / 1e9}), flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"variant": name, "error": str(e)[:200]}), flush=True)
