"""Device CSV ingest probe: where does a 256 MiB chunk's time go? (host read into pinned memory,
H2D, row index + parse kernels, synchronisation) — DeviceTextReader alone, no scoring."""

import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.stream.device_text import DeviceTextReader
    from flink_jpmml_amd.utils.metrics import METRICS

    rows = int(os.environ.get("ROWS", 4 << 20))
    F = 32
    X = synth.stream_matrix(rows, F, seed=1)
    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    path = os.path.join(d, f"probe-{os.getpid()}.csv")
    with open(path, "w") as fh:
        fh.write(",".join(f"f{j}" for j in range(F)) + "\n")
        np.savetxt(fh, X, fmt="%.7g", delimiter=",")
    size = os.path.getsize(path)
    model = CompiledPmml.from_string(synth.gbdt_pmml(n_trees=4, depth=3, n_features=F, seed=1))
    cols = [f"f{j}" for j in range(F)]
    with open(path, "rb") as fh:
        lo = len(fh.readline())
    out = {"bytes": size, "rows": rows}
    configs = [(16, 64 << 20, False), (16, 256 << 20, False), (8, 64 << 20, True), (8, 128 << 20, True),
               (8, 256 << 20, True)]
    for threads, chunk, zc in configs:
        r = DeviceTextReader(path, model, cols, lo, size, torch.device("cuda"), chunk_bytes=chunk, threads=threads,
                             zero_copy=zc)
        first = None
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 0
            for b in r:
                n += len(b)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            first = dt if first is None else first
        out[f"t{threads}_c{chunk >> 20}M_zc{int(zc)}"] = {
            "rows": n, "s": dt, "first_s": first, "zero_copy_active": getattr(r, "zero_copy_active", False),
            "rows_per_s": n / dt, "GBps": (size - lo) / dt / 1e9,
            "timers": {k: v for k, v in METRICS.summary().get("histograms", {}).items() if k.startswith("ingest.")}}
        METRICS.reset()
    # host read alone (pinned), 16 threads
    from concurrent.futures import ThreadPoolExecutor

    buf = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
    fd = os.open(path, os.O_RDONLY)
    pool = ThreadPoolExecutor(16)
    rr = DeviceTextReader(path, model, cols, lo, size, torch.device("cuda"), threads=16)
    t0 = time.perf_counter()
    done = 0
    for a in range(lo, size, 256 << 20):
        b = min(size, a + (256 << 20))
        rr._read(fd, pool, a, b, buf)
        done += b - a
    out["host_read_GBps_16t"] = done / (time.perf_counter() - t0) / 1e9
    dev = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        dev.copy_(buf, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_GBps_1stream"] = 8 * (256 << 20) / (time.perf_counter() - t0) / 1e9
    os.close(fd)
    os.unlink(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
