#!/usr/bin/env python3
"""Headline benchmark: whole-node records/s scoring a 1000-tree GBDT PMML on MI355X (+ p50 latency).

Metric / config from ``BASELINE.json``: "records/sec (whole node) on 1k-tree GBDT PMML at
1/2/4/8 MI355X; p50 latency" — 1000-tree XGBoost-style GBDT PMML (depth 6, 32 float features),
synthetic 1M-row stream per GPU per step (weak scaling), random-initialised trees.

One step (per rank) = score this rank's 1,048,576-row shard end to end:
pinned host records → H2D (copy stream) → fused prepare + tree-ensemble HIP kernel → scores D2H
(pinned host sink), pipelined in micro-batches over three HIP streams; with N > 1 ranks the scored
shards are also all-gathered over RCCL (the stream sink). Nothing is skipped or
cached inside the timed region: every step re-copies and re-scores every row.

Usage::

    python bench.py                                # 1 GPU, defaults
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 3

Rank 0 prints ONE JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

METRIC = "records/sec (whole node) on 1k-tree GBDT PMML at 1/2/4/8 MI355X; p50 latency"


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--trees", type=int, default=1000)
    p.add_argument("--depth", type=int, default=6)
    p.add_argument("--features", type=int, default=32)
    p.add_argument("--rows", type=int, default=1 << 20, help="rows per GPU per step")
    p.add_argument("--micro-batch", type=int, default=1 << 19)
    p.add_argument("--pipeline-depth", type=int, default=3, help="input ring slots (H2D/compute overlap)")
    p.add_argument("--h2d-streams", type=int, default=1, help="concurrent copy streams per micro-batch (1 measured best: splitting adds ~2 ms of host submit per step)")
    p.add_argument("--objective", choices=["regression", "binary"], default="regression",
                   help="binary = modelChain GBDT -> logistic calibrator (BASELINE config 5)")
    p.add_argument("--precision", choices=["fp32", "fp8"], default="fp32",
                   help="leaf-value precision (fp8 = OCP e4m3 leaves, fp32 thresholds; config 5)")
    p.add_argument("--latency-batch", type=int, default=4096)
    p.add_argument("--latency-iters", type=int, default=50)
    p.add_argument("--no-allgather", action="store_true")
    p.add_argument("--check-rows", type=int, default=8192, help="rows checked against the fp64 oracle (untimed)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-numa", action="store_true", help="do not bind to the GPU's NUMA node")
    return p.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    import torch
    import torch.distributed as dist

    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.parallel import all_gather_scores, broadcast_plan, init_from_env
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.engine import StreamingScorer

    if not torch.cuda.is_available():
        print(json.dumps({"metric": METRIC, "error": "no GPU visible"}))
        return 1
    ctx = init_from_env()
    device = ctx.device
    N = ctx.world_size
    if args.gpus != N and ctx.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={N}; using {N}", file=sys.stderr)

    # ---- model: rank 0 generates + parses + lowers once; RCCL-broadcast of the device tensors
    t_load = time.perf_counter()
    compiled = None
    plan = None
    if ctx.rank == 0:
        text = gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, seed=args.seed,
                         objective=args.objective)
        compiled = CompiledPmml.from_string(text)
        plan = compiled.plan(device, precision=args.precision)
    plan = broadcast_plan(plan, ctx)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t_load

    # ---- untimed correctness spot-check against the float64 oracle (rank 0)
    check = {}
    if ctx.rank == 0 and args.check_rows > 0:
        Xc = stream_matrix(args.check_rows, args.features, seed=99, missing_rate=0.02)
        s_ref, v_ref = compiled.score_matrix_oracle(Xc)
        s_gpu, v_gpu = plan.score(Xc)
        s_gpu = s_gpu.cpu().numpy()
        v_gpu = v_gpu.cpu().numpy()
        both = v_ref & v_gpu
        err = float(np.max(np.abs(s_gpu[both] - s_ref[both]))) if both.any() else float("nan")
        check = {"oracle_rows": int(args.check_rows), "valid_match": bool((v_ref == v_gpu).all()),
                 "max_abs_err_vs_fp64": err, "exact_match_rate": float((s_gpu[both] == s_ref[both]).mean())}

    # ---- this rank's synthetic record shard in pinned host memory, on the GPU's NUMA node
    from flink_jpmml_amd.utils.numa import bind_to_gpu_numa

    numa_node = None if args.no_numa else bind_to_gpu_numa(device.index or 0)
    X = torch.from_numpy(stream_matrix(args.rows, args.features, seed=1000 + ctx.rank)).pin_memory()
    score_h = torch.empty(args.rows, dtype=torch.float32).pin_memory()
    valid_h = torch.empty(args.rows, dtype=torch.uint8).pin_memory()
    scorer = StreamingScorer(plan, micro_batch=args.micro_batch, depth=args.pipeline_depth, max_rows=args.rows,
                             h2d_streams=args.h2d_streams)
    gather_out = None
    if N > 1 and not args.no_allgather:
        gather_out = (torch.empty(args.rows * N, dtype=torch.float32, device=device),
                      torch.empty(args.rows * N, dtype=torch.uint8, device=device))

    comm = torch.cuda.Stream(device) if gather_out is not None else None

    def step():
        h = scorer.submit(X, score_h, valid_h)
        if gather_out is not None:
            # all-gather this step's scored shard on a side stream (overlaps the next step)
            comm.wait_stream(scorer.comp)
            with torch.cuda.stream(comm):
                _, _, works = all_gather_scores(h.score_dev, h.valid_dev, ctx, async_op=True, out=gather_out)
                for w in works:
                    w.wait()
            scorer.mark_consumed(h, comm)
        return h

    for _ in range(args.warmup):
        scorer.wait(step())
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = None
    host_submit = 0.0
    for _ in range(args.steps):
        ts = time.perf_counter()
        h = step()
        host_submit += time.perf_counter() - ts
    scorer.wait(h)
    scorer.join()
    if comm is not None:
        torch.cuda.current_stream().wait_stream(comm)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ctx.is_distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    records_per_s = N * args.rows * args.steps / elapsed

    # ---- device-resident kernel throughput (records already in HBM) — reported separately
    Xd = X[: args.rows].to(device)
    sd = torch.empty(args.rows, dtype=torch.float32, device=device)
    vd = torch.empty(args.rows, dtype=torch.uint8, device=device)
    for _ in range(2):
        plan.launch(Xd, sd, vd)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kiters = 5
    e0.record()
    for _ in range(kiters):
        plan.launch(Xd, sd, vd)
    e1.record()
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1) / kiters

    # ---- p50 latency: one micro-batch end to end (host records -> host scores), unpipelined
    lat_scorer = StreamingScorer(plan, micro_batch=args.latency_batch, depth=1, max_rows=args.latency_batch)
    Xl = torch.from_numpy(stream_matrix(args.latency_batch, args.features, seed=7)).pin_memory()
    sl = torch.empty(args.latency_batch, dtype=torch.float32).pin_memory()
    vl = torch.empty(args.latency_batch, dtype=torch.uint8).pin_memory()
    lats = []
    for i in range(args.latency_iters + 5):
        t1 = time.perf_counter()
        lat_scorer.wait(lat_scorer.submit(Xl, sl, vl))
        if i >= 5:
            lats.append((time.perf_counter() - t1) * 1e3)
    p50 = float(np.percentile(lats, 50))
    p99 = float(np.percentile(lats, 99))

    if ctx.rank == 0:
        out = {
            "metric": METRIC,
            "value": records_per_s,
            "unit": "records/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.precision == "fp32" else "fp32 (fp8 e4m3 leaf values)",
            "data": "synthetic (random-init XGBoost-style GBDT PMML, N(0,1) float records)",
            "config": {
                "model": f"GBDT {args.trees} trees, depth {args.depth}, {args.features} float features "
                         f"(XGBoost-style PMML, {args.objective}, {args.precision} leaves)",
                "global_batch": args.rows * N,
                "seq_len": None,
                "parallelism": f"dp{N}",
                "micro_batch": args.micro_batch,
                "pipeline_depth": args.pipeline_depth,
                "h2d_streams": args.h2d_streams,
                "rows_per_gpu_per_step": args.rows,
                "allgather_sink": bool(gather_out is not None),
                "zero_copy_host_sink": bool(scorer.direct),
                "numa_node": numa_node,
            },
            "p50_latency_ms": p50,
            "p99_latency_ms": p99,
            "latency_batch_rows": args.latency_batch,
            "kernel_only_records_per_s_per_gpu": args.rows / (kernel_ms / 1e3),
            "kernel_ms_per_1M_rows": kernel_ms * (1 << 20) / args.rows,
            "model_load_broadcast_s": load_s,
            "host_submit_ms_per_step": host_submit / args.steps * 1e3,
            "plan": {"layout": getattr(plan, "layout", None), "depth": getattr(plan, "depth", None),
                     "chunk_trees": getattr(plan, "chunk_trees", None)},
            "check": check,
        }
        print(json.dumps(out), flush=True)
    if ctx.is_distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
