"""Probe: host->device ingest bandwidth on one MI355X for the bench's 1M x 32 fp32 step (128 MiB).

* SDMA copies: one stream, and the same bytes split over 2 / 4 streams;
* kernel pull: CUs read the pinned buffer through its device-visible address (pmml_pull_copy);
* fused pull: the tree kernel reads its records straight from pinned host memory (no copy stage).
Prints one JSON line of GB/s (and ms per 1M-row step for the fused mode)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.ops import _lib  # noqa: E402
from flink_jpmml_amd.runtime.compiled import CompiledPmml  # noqa: E402

ROWS, F, IT = 1 << 20, 32, 10
lib = _lib.load()
lib.pmml_pull_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
lib.pmml_pull_copy.restype = ctypes.c_int
Xh = torch.from_numpy(stream_matrix(ROWS, F, seed=1)).pin_memory()
Xd = torch.empty_like(Xh, device="cuda")
nbytes = Xh.numel() * 4
res = {"bytes": nbytes}


def timeit(fn, iters=IT):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


for k in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(k)]
    rows = ROWS // k

    def copy_k():
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                Xd[i * rows:(i + 1) * rows].copy_(Xh[i * rows:(i + 1) * rows], non_blocking=True)
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)

    res[f"sdma_{k}stream_GBps"] = nbytes / timeit(copy_k) / 1e9

hdev = _lib.host_device_ptr(Xh)
st = torch.cuda.current_stream().cuda_stream
for blocks in (256, 1024, 4096):
    t = timeit(lambda: _lib.check(lib.pmml_pull_copy(st, hdev, Xd.data_ptr(), nbytes, blocks), "pull"))
    res[f"pull_{blocks}blk_GBps"] = nbytes / t / 1e9

c = CompiledPmml.from_string(gbdt_pmml(n_trees=1000, depth=6, n_features=F))
plan = c.plan("cuda:0")
sd = torch.empty(ROWS, device="cuda")
vd = torch.empty(ROWS, dtype=torch.uint8, device="cuda")
res["kernel_device_ms"] = timeit(lambda: plan.launch(Xd, sd, vd)) * 1e3


class HostView:  # a tensor-like wrapper whose data_ptr is the device-visible host address
    shape = (ROWS, F)

    def data_ptr(self):
        return hdev

    def stride(self, i):
        return F if i == 0 else 1


res["kernel_fused_pull_ms"] = timeit(lambda: plan.launch(HostView(), sd, vd)) * 1e3
s_ref = sd.clone()
plan.launch(Xd, sd, vd)
torch.cuda.synchronize()
res["fused_pull_matches"] = bool(torch.equal(s_ref, sd))
print(json.dumps(res))
