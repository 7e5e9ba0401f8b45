#!/usr/bin/env python3
"""Can one host feed 8 GPUs x ~56 GB/s of pinned-buffer H2D?

On the 1-GPU box: (A) H2D of a 1 GiB pinned buffer alone (the bench's path: this process bound to
the GPU's NUMA node); (B) 8 concurrent reader processes (``numa_read_probe.cpp``), each bound to a
NUMA node round-robin and streaming its own locally first-touched buffer — the host DRAM read
bandwidth 8 ranks' ingest threads / DMA engines would compete for; (C) 7 readers + the H2D at
once. One JSON object on stdout."""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def nodes():
    base = "/sys/devices/system/node"
    out = []
    allowed = os.sched_getaffinity(0)
    from flink_jpmml_amd.utils.numa import _parse_cpulist

    for d in sorted(os.listdir(base)):
        if d.startswith("node") and d[4:].isdigit():
            with open(os.path.join(base, d, "cpulist")) as fh:
                if set(_parse_cpulist(fh.read())) & allowed:
                    out.append(int(d[4:]))
    return out or [0]


def h2d(seconds):
    import torch

    x = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    y = torch.empty_like(x, device="cuda")
    y.copy_(x, non_blocking=True)
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        y.copy_(x, non_blocking=True)
        torch.cuda.synchronize()
        n += 1
    return n * x.numel() / (time.perf_counter() - t0) / 1e9


def readers(exe, k, threads, mib, seconds, ns):
    procs = [subprocess.Popen([exe, str(ns[i % len(ns)]), str(threads), str(mib), str(seconds)],
                              stdout=subprocess.PIPE, text=True) for i in range(k)]
    return procs


def collect(procs):
    out = []
    for p in procs:
        o, _ = p.communicate(timeout=120)
        out.append(json.loads(o.strip().splitlines()[-1]))
    return out


def main():
    exe = os.path.join("/tmp", "numa_read_probe")
    subprocess.run(["g++", "-O3", "-march=x86-64-v3", "-pthread", "-o", exe,
                    os.path.join(HERE, "numa_read_probe.cpp")], check=True)
    from flink_jpmml_amd.utils.numa import bind_to_gpu_numa

    ns = nodes()
    gpu_node = bind_to_gpu_numa(0)
    res = {"numa_nodes_allowed": ns, "gpu_numa_node": gpu_node, "cpus_allowed": len(os.sched_getaffinity(0)),
           "cpu_count": os.cpu_count()}
    res["A_h2d_alone_gbps"] = h2d(3.0)
    r = collect(readers(exe, 8, 2, 1024, 4, ns))
    res["B_8_readers"] = r
    res["B_8_readers_total_gbps"] = sum(x["gbps"] for x in r)
    procs = readers(exe, 7, 2, 1024, 6, ns)
    time.sleep(1.0)
    res["C_h2d_with_7_readers_gbps"] = h2d(3.0)
    r = collect(procs)
    res["C_7_readers_total_gbps"] = sum(x["gbps"] for x in r)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
