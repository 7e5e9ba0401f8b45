#!/usr/bin/env python3
"""Headline benchmark: whole-node records/s scoring a 1000-tree GBDT PMML on MI355X (+ p50 latency).

Metric / config from ``BASELINE.json``: "records/sec (whole node) on 1k-tree GBDT PMML at
1/2/4/8 MI355X; p50 latency" — 1000-tree XGBoost-style GBDT PMML (depth 6, 32 float features),
synthetic record stream, random-initialised trees (weak scaling: each GPU scores its own shard).

**The timed path is the public DSL** (``--api dsl``, default)::

    env = StreamExecutionEnvironment(config=ScoringConfig(device="cuda", ...), dist_ctx=ctx)
    env.add_source(<pinned RecordBatch per step>, mode="parallel")
       .quick_evaluate(ModelReader(model.pmml))            # EvaluationFunction, one per rank
       .add_sink(<waits for every PredictionBatch; all-gathers the scores over RCCL when N > 1>)

One step (per rank) = ``--passes`` RecordBatches of ``--rows`` records each (passes over this
rank's pinned shard) scored end to end: H2D in micro-batches on a copy stream → fused prepare +
tree-ensemble HIP kernel whose epilogue writes scores straight into pinned host memory → the
library :class:`~flink_jpmml_amd.parallel.sinks.GatherSink` (lockstep) waits for every batch and,
with N > 1, all-gathers the scored shard's device mirrors over RCCL on a comm stream (SURVEY §2.6
F5). Nothing is skipped or cached: every pass re-copies and re-scores every row (a step is
``passes × rows`` records, so the timed region is seconds long). ``--api engine`` times the bare
StreamingScorer instead.

Under ``torchrun`` the model is parsed once on rank 0 and its compiled tensors are
RCCL-broadcast to every rank (F2). Rank 0 prints ONE JSON line.

    python bench.py                                # 1 GPU, defaults
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 3
    python bench.py --model rf|chain|mlp           # BASELINE configs 3 / 5 / 4
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

METRIC = "records/sec (whole node) on 1k-tree GBDT PMML at 1/2/4/8 MI355X; p50 latency"

MODELS = {
    # name: (BASELINE config, description)
    "gbdt": ("1000-tree GBDT PMML (XGBoost-exported), 1M-row synthetic stream, 1xMI355X", "GBDT regression"),
    "chain": ("MiningModel ensemble (GBDT chain + logistic calibrator), fp8 weights on CDNA4",
              "GBDT modelChain -> logistic calibrator"),
    "rf": ("500-tree RandomForest PMML, DP=8 stream shard over xGMI on 8xMI355X", "random forest majority vote"),
    "mlp": ("3-layer NeuralNetwork PMML, bf16 MFMA GEMM path, 8xMI355X", "NeuralNetwork 64-256-256-1"),
}


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--api", choices=["dsl", "engine"], default="dsl")
    p.add_argument("--source", choices=["synthetic", "binary", "text"], default="synthetic",
                   help="synthetic: pinned in-memory shard (headline); binary: memory-mapped fp32 record file "
                        "(zero-parse ingest); text: CSV through the native parser -- reported separately")
    p.add_argument("--ingest-threads", type=int, default=8, help="binary copy / text parse threads per rank")
    p.add_argument("--model", choices=sorted(MODELS), default="gbdt")
    p.add_argument("--trees", type=int, default=None, help="default 1000 (gbdt/chain), 500 (rf)")
    p.add_argument("--depth", type=int, default=None, help="default 6 (gbdt/chain), 8 (rf)")
    p.add_argument("--features", type=int, default=None, help="default 32 (trees), 64 (mlp)")
    p.add_argument("--rows", type=int, default=1 << 23,
                   help="rows per pass (this rank's pinned shard: 8M rows x 32 fp32 = 1 GiB)")
    p.add_argument("--passes", type=int, default=16,
                   help="passes over the pinned shard per step (16: a 20-step timed region is ~6 s on one GPU)")
    p.add_argument("--micro-batch", type=int, default=1 << 20,
                   help="rows per H2D slice + kernel launch (1M measured best: profiles/r2_h2d_probe.md)")
    p.add_argument("--pipeline-depth", type=int, default=3, help="input ring slots (H2D/compute overlap)")
    p.add_argument("--h2d-streams", type=int, default=0,
                   help="copy streams per micro-batch (copy engines); 0 = calibrate 1 vs 2 on this box")
    p.add_argument("--max-inflight", type=int, default=3, help="scored steps in flight before the sink waits")
    p.add_argument("--precision", choices=["fp32", "bf16", "fp8"], default=None,
                   help="default fp32 (trees), bf16 (mlp, BASELINE config 4); fp8 = e4m3 leaves (config 5)")
    p.add_argument("--latency-batch", type=int, default=4096)
    p.add_argument("--latency-iters", type=int, default=50)
    p.add_argument("--no-allgather", action="store_true")
    p.add_argument("--check-rows", type=int, default=8192, help="rows checked against the fp64 oracle (untimed)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-numa", action="store_true", help="do not bind to the GPU's NUMA node")
    p.add_argument("--force-dist", action="store_true", help="form a 1-rank RCCL group at N=1 (exercise RCCL)")
    a = p.parse_args(argv)
    a.trees = a.trees or (500 if a.model == "rf" else 1000)
    a.depth = a.depth or (8 if a.model == "rf" else 6)
    a.features = a.features or (64 if a.model == "mlp" else 32)
    a.precision = a.precision or ("bf16" if a.model == "mlp" else "fp32")
    return a


def model_text(args) -> str:
    from flink_jpmml_amd.bench import synth

    if args.model == "gbdt":
        return synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, seed=args.seed)
    if args.model == "chain":
        return synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, seed=args.seed,
                               objective="binary")
    if args.model == "rf":
        return synth.random_forest_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features,
                                        n_classes=3, seed=args.seed)
    return synth.mlp_pmml(n_features=args.features, hidden=(256, 256), n_out=1, seed=args.seed)


class _StepSource:
    """``--warmup + --steps`` RecordBatches (one per step) of this rank's pinned shard; calls
    ``on_step(i)`` right before step i is handed to the pipeline (timer start hook)."""

    def __init__(self, X, n_steps, passes, on_step):
        self.X = X
        self.n = n_steps
        self.passes = passes
        self.on_step = on_step

    def open_subtask(self, rank, world):  # parallel source: every rank scores its own shard
        pass

    def iterate(self):
        from flink_jpmml_amd.api.batch import RecordBatch

        rows = len(self.X)
        for i in range(self.n):
            self.on_step(i)
            for p in range(self.passes):
                yield RecordBatch(self.X, offset=(i * self.passes + p) * rows)


class _FileStepSource:
    """``--source binary|text``: every step reads this rank's record file ``passes`` times through
    the library's file source (binary: mmap + parallel copy into pinned buffers; text: the native
    multi-threaded parser into pinned buffers); ``on_step(i)`` fires at step boundaries."""

    def __init__(self, make_source, n_steps, passes, on_step):
        self.make_source = make_source
        self.n = n_steps
        self.passes = passes
        self.on_step = on_step

    def open_subtask(self, rank, world):
        pass

    def iterate(self):
        off = 0
        for i in range(self.n):
            self.on_step(i)
            for _ in range(self.passes):
                for b in self.make_source().iterate():
                    b.offset = off
                    off += len(b)
                    yield b


def _write_source_file(args, X, rank):
    """This rank's record file for ``--source binary|text`` (page-cache resident after writing)."""
    import tempfile

    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    if args.source == "binary":
        from flink_jpmml_amd.stream.binary import write_binary

        return write_binary(os.path.join(d, f"fja-bench-{os.getpid()}-{rank}.fjab"), X)
    path = os.path.join(d, f"fja-bench-{os.getpid()}-{rank}.csv")
    with open(path, "w") as fh:
        fh.write(",".join(f"f{j}" for j in range(X.shape[1])) + "\n")
        np.savetxt(fh, X, fmt="%.7g", delimiter=",")
    return path


class _WaitSink:
    """``--no-allgather`` at N > 1: every rank only waits for its own scored batches."""

    def __init__(self):
        self.rows_seen = 0

    def invoke(self, value) -> None:
        value[0].wait()
        self.rows_seen += len(value[0])

    def finish(self) -> None:
        pass


def _h2d_streams(pipe, args):
    """Copy streams of the pipeline the timed operator used (auto mode: its calibration's choice)."""
    n = getattr(pipe, "h2d_streams_in_use", None) if pipe is not None else None
    return int(n) if n else (args.h2d_streams or None)


def main(argv=None) -> int:
    args = parse_args(argv)
    import torch
    import torch.distributed as dist

    from flink_jpmml_amd import ModelReader
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.parallel import broadcast_object, init_from_env
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.engine import StreamingScorer
    from flink_jpmml_amd.runtime.loading import load_replicated
    from flink_jpmml_amd.utils.metrics import METRICS

    if not torch.cuda.is_available():
        print(json.dumps({"metric": METRIC, "error": "no GPU visible"}))
        return 1
    ctx = init_from_env(force=args.force_dist)
    device = ctx.device
    N = ctx.world_size
    if args.gpus != N and ctx.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={N}; using {N}", file=sys.stderr)
    cfg = ScoringConfig(device=device, micro_batch=args.micro_batch, pipeline_depth=args.pipeline_depth,
                        max_inflight=args.max_inflight, precision=args.precision, fallback="error",
                        h2d_streams=args.h2d_streams)

    # ---- the model: rank 0 writes the synthetic PMML; every rank loads it through the collective
    #      parse-once / RCCL-broadcast path the DSL operators use
    path = None
    if ctx.rank == 0:
        fd, path = tempfile.mkstemp(suffix=".pmml", prefix="bench-")
        with os.fdopen(fd, "w") as fh:
            fh.write(model_text(args))
    path = broadcast_object(path, ctx)
    t_load = time.perf_counter()
    lm = load_replicated(path, ctx, device, cfg)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t_load
    model = lm.model
    plan = model.scorer.plan

    # ---- untimed correctness spot-check against the float64 oracle (rank 0)
    check = {}
    if ctx.rank == 0 and args.check_rows > 0:
        compiled = CompiledPmml.from_string(open(path).read())
        Xc = stream_matrix(args.check_rows, args.features, seed=99, missing_rate=0.02)
        s_ref, v_ref = compiled.score_matrix_oracle(Xc)
        pb = model.predict(Xc)
        s_gpu, v_gpu = pb.scores, pb.valid
        both = v_ref & v_gpu
        err = float(np.max(np.abs(s_gpu[both] - s_ref[both]))) if both.any() else float("nan")
        check = {"oracle_rows": int(args.check_rows), "valid_match": bool((v_ref == v_gpu).all()),
                 "max_abs_err_vs_fp64": err, "exact_match_rate": float((s_gpu[both] == s_ref[both]).mean())}

    # ---- this rank's synthetic record shard in pinned host memory, on the GPU's NUMA node
    from flink_jpmml_amd.utils.numa import bind_to_gpu_numa

    numa_node = None if args.no_numa else bind_to_gpu_numa(device.index or 0)
    X = torch.from_numpy(stream_matrix(args.rows, args.features, seed=1000 + ctx.rank)).pin_memory()
    # every distributed run all-gathers (a 1-rank RCCL group under --force-dist takes the same
    # device-mirror / RCCL path as N > 1)
    gather = ctx.is_distributed and not args.no_allgather
    timing = {}

    def barrier_sync():
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()

    pipe = None
    job = {}
    rows_per_step = args.rows * args.passes
    if args.api == "dsl":
        from flink_jpmml_amd.parallel.sinks import GatherSink
        from flink_jpmml_amd.stream import StreamExecutionEnvironment

        def on_step(i):
            if i == args.warmup:
                barrier_sync()
                timing["t0"] = time.perf_counter()

        env = StreamExecutionEnvironment(config=cfg, dist_ctx=ctx if ctx.is_distributed else None)
        # the library F5 sink: waits for every scored batch; with N > 1 all-gathers the device
        # mirrors over RCCL on its comm stream, overlapping the next batch
        sink = GatherSink(to="all", lockstep=True, keep=False) if gather or not ctx.is_distributed else _WaitSink()
        op_cfg = cfg.replace(device_mirror=gather)
        if args.source == "synthetic":
            src = _StepSource(X, args.warmup + args.steps, args.passes, on_step)
        else:
            from flink_jpmml_amd.stream.binary import BinaryBatchSource
            from flink_jpmml_amd.stream.sources import TextBatchSource

            src_path = _write_source_file(args, X.numpy(), ctx.rank)
            job["source_file_bytes"] = os.path.getsize(src_path)
            if args.source == "binary":
                make = lambda: BinaryBatchSource(src_path, batch_rows=args.micro_batch,  # noqa: E731
                                                 threads=args.ingest_threads)
            else:
                text_model = CompiledPmml.load(path)  # parsed once: field names + vocabularies
                make = lambda: TextBatchSource(src_path, text_model, batch_rows=args.micro_batch,  # noqa: E731
                                               threads=args.ingest_threads)
            src = _FileStepSource(make, args.warmup + args.steps, args.passes, on_step)
        stream = env.add_source(src, mode="parallel")
        scored = stream.quick_evaluate(ModelReader(path), config=op_cfg)
        scored.add_sink(sink)
        res = env.execute("bench")
        sink.finish()
        barrier_sync()
        elapsed = time.perf_counter() - timing["t0"]
        job.update(records_in=res.records_in, elements_in=res.elements_in)
        seen = sink.rows_seen
        assert seen == (args.warmup + args.steps) * rows_per_step, (seen, rows_per_step)
        assert res.records_in == seen
        op = scored.node.factory  # the operator instance this (single-subtask) rank ran
        pipe = getattr(getattr(op, "inner", op), "_pipeline", None)
        if args.source != "synthetic":
            os.unlink(src_path)
    else:
        scorer = StreamingScorer(plan, micro_batch=args.micro_batch, depth=args.pipeline_depth, max_rows=args.rows,
                                 h2d_streams=args.h2d_streams)
        pipe = scorer.pipe
        score_h = torch.empty(args.rows, dtype=torch.float32).pin_memory()
        valid_h = torch.empty(args.rows, dtype=torch.uint8).pin_memory()
        for _ in range(args.warmup * args.passes):
            scorer.wait(scorer.submit(X, score_h, valid_h))
        barrier_sync()
        t0 = time.perf_counter()
        h = None
        for _ in range(args.steps * args.passes):
            h = scorer.submit(X, score_h, valid_h)
        scorer.wait(h)
        barrier_sync()
        elapsed = time.perf_counter() - t0
    if ctx.is_distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    records_per_s = N * rows_per_step * args.steps / elapsed

    # ---- device-resident kernel throughput (records already in HBM) — reported separately
    n_k = min(args.rows, 1 << 22)
    Xd = X[:n_k].to(device)
    sd = torch.empty(n_k, dtype=torch.float32, device=device)
    vd = torch.empty(n_k, dtype=torch.uint8, device=device)
    for _ in range(2):
        plan.launch(Xd, sd, vd)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kiters = 10
    e0.record()
    for _ in range(kiters):
        plan.launch(Xd, sd, vd)
    e1.record()
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1) / kiters

    # ---- p50 latency: one small RecordBatch through model.predict (host records -> host scores)
    from flink_jpmml_amd.api.batch import RecordBatch

    Xl = RecordBatch(torch.from_numpy(stream_matrix(args.latency_batch, args.features, seed=7)).pin_memory())
    lats = []
    for i in range(args.latency_iters + 5):
        t1 = time.perf_counter()
        model.predict(Xl).wait()
        if i >= 5:
            lats.append((time.perf_counter() - t1) * 1e3)
    p50 = float(np.percentile(lats, 50))
    p99 = float(np.percentile(lats, 99))

    if ctx.rank == 0:
        default = args.model == "gbdt" and args.source == "synthetic"
        metric = METRIC if default else f"records/sec (whole node) on {MODELS[args.model][1]} PMML; p50 latency"
        if args.source != "synthetic":
            metric += f" [source: {args.source} record file, end to end incl. ingest]"
        out = {
            "metric": metric,
            "value": records_per_s,
            "unit": "records/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"fp32": "fp32", "bf16": "bf16", "fp8": "fp32 (fp8 e4m3 leaf values)"}[args.precision],
            "data": "synthetic (random-init PMML model, N(0,1) float records)" + (
                "" if args.source == "synthetic" else f", read from a {args.source} record file per rank"),
            "config": {
                "model": (f"GBDT {args.trees} trees, depth {args.depth}, {args.features} float features "
                          f"(XGBoost-style PMML, regression, {args.precision} leaves)") if default else
                         f"{MODELS[args.model][1]}: trees={args.trees} depth={args.depth} "
                         f"features={args.features} precision={args.precision}",
                "baseline_config": MODELS[args.model][0],
                "global_batch": rows_per_step * N,
                "seq_len": None,
                "parallelism": f"dp{N}",
                "api": args.api,
                "source": args.source,
                "micro_batch": args.micro_batch,
                "pipeline_depth": args.pipeline_depth,
                "h2d_streams": _h2d_streams(pipe, args),
                "rows_per_gpu_per_step": rows_per_step,
                "passes_per_step": args.passes,
                "rows_per_pass": args.rows,
                "allgather_sink": gather,
                "zero_copy_host_sink": bool(getattr(model.scorer, "direct", False)),
                "numa_node": numa_node,
            },
            "p50_latency_ms": p50,
            "p99_latency_ms": p99,
            "latency_batch_rows": args.latency_batch,
            "kernel_only_records_per_s_per_gpu": n_k / (kernel_ms / 1e3),
            "kernel_ms_per_1M_rows": kernel_ms * (1 << 20) / n_k,
            "h2d_gbps_effective": rows_per_step * args.features * 4 * args.steps / elapsed / 1e9,
            "job": job,
            "model_load_broadcast_s": load_s,
            "timed_region_s": elapsed,
            "plan": {"layout": getattr(plan, "layout", None), "depth": getattr(plan, "depth", None),
                     "chunk_trees": getattr(plan, "chunk_trees", None), "kind": getattr(plan, "kind", None)},
            "check": check,
            "metrics": {k: v for k, v in METRICS.summary()["counters"].items() if not k.startswith("model_cache")},
        }
        print(json.dumps(out), flush=True)
        try:
            os.unlink(path)
        except OSError:
            pass
    if ctx.is_distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
