"""Probe: are pinned H2D copies asynchronous w.r.t. the host? (torch copy_ vs raw hipMemcpyAsync)"""
import ctypes
import json
import time

import torch

n = 16 << 20  # 16 MiB
src = torch.empty(n // 4, dtype=torch.float32).pin_memory()
dst = torch.empty(n // 4, dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
res = {"is_pinned": src.is_pinned()}
for name in ("torch_copy", "torch_copy_slice"):
    times = []
    for i in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            if name == "torch_copy":
                dst.copy_(src, non_blocking=True)
            else:
                dst[: n // 8].copy_(src[n // 8: n // 4], non_blocking=True)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        times.append(((t1 - t0) * 1e6, (t2 - t0) * 1e6))
    res[name] = {"call_us": sorted(t[0] for t in times)[5], "total_us": sorted(t[1] for t in times)[5]}
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
times = []
for i in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), n, 1, s.cuda_stream)
    t1 = time.perf_counter()
    s.synchronize()
    t2 = time.perf_counter()
    times.append(((t1 - t0) * 1e6, (t2 - t0) * 1e6, rc))
res["hipMemcpyAsync"] = {"call_us": sorted(t[0] for t in times)[5], "total_us": sorted(t[1] for t in times)[5],
                         "rc": times[0][2]}
# host-registered (not hipHostMalloc) memory
import numpy as np
a = np.empty(n // 4, dtype=np.float32)
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
rc = hip.hipHostRegister(a.ctypes.data, n, 0)
times = []
for i in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hip.hipMemcpyAsync(dst.data_ptr(), a.ctypes.data, n, 1, s.cuda_stream)
    t1 = time.perf_counter()
    s.synchronize()
    t2 = time.perf_counter()
    times.append(((t1 - t0) * 1e6, (t2 - t0) * 1e6))
res["hostRegister+hipMemcpyAsync"] = {"register_rc": rc, "call_us": sorted(t[0] for t in times)[5],
                                      "total_us": sorted(t[1] for t in times)[5]}
print(json.dumps(res))
