#!/usr/bin/env python3
"""HBM write / copy ceilings for the store-bound first MLP layer: 2 GiB bf16 written by fill_
(write-only) and by copy_ (read + write), CUDA-event timed."""
import json

import torch


def main():
    n = 1 << 30  # bf16 elements = 2 GiB
    a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    out = {}
    for name, fn, nbytes in (("fill", lambda: a.fill_(1.0), 2 * n), ("copy", lambda: b.copy_(a), 4 * n)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        out[name] = {"ms": ms, "TBps": nbytes / ms / 1e9}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
