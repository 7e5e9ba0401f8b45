#!/usr/bin/env python3
"""H2D ceiling: SDMA copies (1 / 2 streams) vs kernel pull (CUs read pinned host memory through its
device-visible address), 128 MiB and 1 GiB pinned buffers on the GPU's NUMA node."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.ops import _lib
    from flink_jpmml_amd.utils.numa import bind_to_gpu_numa

    lib = _lib.load()
    lib.pmml_pull_copy.restype = ctypes.c_int
    lib.pmml_pull_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    node = bind_to_gpu_numa(0)
    res = {"numa": node}
    for mib in (128, 1024):
        n = mib << 20
        src = torch.empty(n // 4, dtype=torch.float32).pin_memory()
        src.fill_(1.0)
        dst = torch.empty(n // 4, dtype=torch.float32, device="cuda")
        dev_src = _lib.host_device_ptr(src)
        streams = [torch.cuda.Stream() for _ in range(2)]

        def timed(fn, reps=5):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return n * reps / (time.perf_counter() - t0) / 1e9

        def sdma(k):
            def fn():
                part = n // k
                for j in range(k):
                    lib.pmml_memcpy_async(dst.data_ptr() + j * part, src.data_ptr() + j * part, part, 1,
                                          streams[j].cuda_stream)
            return fn

        res[f"{mib}MiB_sdma1_GBps"] = timed(sdma(1))
        res[f"{mib}MiB_sdma2_GBps"] = timed(sdma(2))
        if dev_src:
            for blocks in (256, 1024, 2048, 4096):
                res[f"{mib}MiB_pull{blocks}_GBps"] = timed(
                    lambda b=blocks: lib.pmml_pull_copy(streams[0].cuda_stream, dev_src, dst.data_ptr(), n, b))
            assert bool((dst == 1.0).all())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
