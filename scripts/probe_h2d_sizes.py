"""Probe: pinned host -> device copy bandwidth vs buffer size and NUMA placement.

Measures one-stream H2D of 512K-row (64 MiB at 32 fp32 features) slices cycling through a pinned
buffer of ``--rows`` rows, the pattern of the engine's input ring. Run once per placement (the
binding must happen before the pinned allocation). Prints one JSON line.

    python scripts/probe_h2d_sizes.py --rows 8388608 [--numa auto|none|<node>]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=1 << 20)
    p.add_argument("--features", type=int, default=32)
    p.add_argument("--slice", type=int, default=1 << 19)
    p.add_argument("--numa", default="auto")
    p.add_argument("--passes", type=int, default=4)
    a = p.parse_args()
    import torch

    from flink_jpmml_amd.utils.numa import _parse_cpulist, bind_to_gpu_numa, gpu_numa_node

    node = None
    if a.numa == "auto":
        node = bind_to_gpu_numa(0)
    elif a.numa != "none":
        with open(f"/sys/devices/system/node/node{int(a.numa)}/cpulist") as fh:
            os.sched_setaffinity(0, set(_parse_cpulist(fh.read())))
        node = int(a.numa)
    X = torch.empty((a.rows, a.features), dtype=torch.float32, pin_memory=True)
    X.fill_(1.0)  # first touch on this node
    slots = [torch.empty((a.slice, a.features), dtype=torch.float32, device="cuda") for _ in range(3)]
    st = torch.cuda.Stream()
    n_sl = a.rows // a.slice

    def one_pass():
        with torch.cuda.stream(st):
            for i in range(n_sl):
                slots[i % 3].copy_(X[i * a.slice:(i + 1) * a.slice], non_blocking=True)

    one_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.passes):
        one_pass()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gb = a.rows * a.features * 4 * a.passes / 1e9
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))
    print(json.dumps({"rows": a.rows, "numa": a.numa, "bound_node": node, "gpu_node": gpu_numa_node(0),
                      "nodes": nodes, "cpus": len(os.sched_getaffinity(0)), "h2d_GBps": gb / dt,
                      "slice_rows": a.slice}), flush=True)


if __name__ == "__main__":
    main()
