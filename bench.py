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
    python bench.py --gpus 8 --steps 20 --warmup 3   # spawns the 8 ranks itself (launch_ranks)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 3   # same job, external launcher
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
    p.add_argument("--models", type=int, default=1,
                   help="> 1: dynamic serving of this many models (AddMessage control stream); every record "
                        "names a random one (dictionary-encoded model_ids) and each pass is scored through "
                        "ConnectedStreams.quick_evaluate's grouped device pass")
    p.add_argument("--rehearse-cpu", action="store_true",
                   help="run the exact DSL / sink / collective code on the CPU (host oracle scorer, gloo): a "
                        "functional rehearsal of N ranks without GPUs -- its numbers are NOT a benchmark")
    p.add_argument("--model-docs", type=int, default=8,
                   help="--models mode: distinct synthetic PMML documents (seeds) the model ids cycle over")
    a = p.parse_args(argv)
    a.trees = a.trees or (500 if a.model == "rf" else 1000)
    a.depth = a.depth or (8 if a.model == "rf" else 6)
    a.features = a.features or (64 if a.model == "mlp" else 32)
    a.precision = a.precision or ("bf16" if a.model == "mlp" else "fp32")
    return a


def model_text(args, seed=None) -> str:
    from flink_jpmml_amd.bench import synth

    seed = args.seed if seed is None else seed
    if args.model == "gbdt":
        return synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, seed=seed)
    if args.model == "chain":
        return synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, seed=seed,
                               objective="binary")
    if args.model == "rf":
        return synth.random_forest_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features,
                                        n_classes=3, seed=seed)
    return synth.mlp_pmml(n_features=args.features, hidden=(256, 256), n_out=1, seed=seed)


class _StepSource:
    """``--warmup + --steps`` RecordBatches (one per step) of this rank's pinned shard; calls
    ``on_step(i)`` right before step i is handed to the pipeline (timer start hook). ``model_ids``
    (``--models`` mode): the per-row ``(codes, ids)`` column every batch carries."""

    def __init__(self, X, n_steps, passes, on_step, model_ids=None):
        self.X = X
        self.n = n_steps
        self.passes = passes
        self.on_step = on_step
        self.model_ids = model_ids

    def open_subtask(self, rank, world):  # parallel source: every rank scores its own shard
        pass

    def iterate(self):
        from flink_jpmml_amd.api.batch import RecordBatch

        rows = len(self.X)
        for i in range(self.n):
            self.on_step(i)
            for p in range(self.passes):
                yield RecordBatch(self.X, model_ids=self.model_ids, offset=(i * self.passes + p) * rows)


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


def _kernel_ms(plan, Xh, device) -> float:
    """Kernel-only time of one launch over the device-resident rows ``Xh`` (ms)."""
    import torch

    n_k = Xh.shape[0]
    Xd = Xh.to(device)
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
    return e0.elapsed_time(e1) / kiters


def _rehearsal_reference(args, rank, doc_paths):
    """``(scores, valid)`` this rank's records must score to (CPU rehearsal): the fp64 oracle of the
    model each record names over the records this rank's source produced."""
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    X = stream_matrix(args.rows, args.features, seed=1000 + rank)
    if args.source == "text":  # what the CSV the rank wrote holds (%.7g), parsed back
        import io

        buf = io.StringIO()
        np.savetxt(buf, X, fmt="%.7g", delimiter=",")
        X = np.loadtxt(io.StringIO(buf.getvalue()), delimiter=",", dtype=np.float64).reshape(X.shape)
    X = X.astype(np.float32)
    docs = [CompiledPmml.from_string(open(p).read()) for p in doc_paths]
    if args.models <= 1:
        return docs[0].score_matrix_oracle(X)
    codes = np.random.default_rng(2000 + rank).integers(0, args.models, args.rows)
    s = np.full(args.rows, np.nan)
    v = np.zeros(args.rows, dtype=bool)
    for k in np.unique(codes).tolist():
        rows = np.flatnonzero(codes == k)
        s[rows], v[rows] = docs[k % len(docs)].score_matrix_oracle(X[rows])
    return s, v


def _rehearsal_check(args, sink, ctx, doc_paths):
    """Every gathered element holds the N ranks' equal-size chunks in rank order; this rank's chunk
    must be its records in source order (consecutive offsets) scoring like its reference."""
    ref_s, ref_v = _rehearsal_reference(args, ctx.rank, doc_paths)
    ref_s = ref_s.astype(np.float32)
    N, me = ctx.world_size, ctx.rank
    ok, checked, expect_off = True, 0, 0
    tol = 1e-5 if args.source == "text" else 0.0  # CSV: decimal -> float32 rounding may differ per parser
    for s, v, o in sink._parts:
        if len(s) % N:
            return False, checked
        m = len(s) // N
        cs, cv, co = s[me * m:(me + 1) * m], v[me * m:(me + 1) * m], o[me * m:(me + 1) * m]
        ok = ok and bool((co == expect_off + np.arange(m)).all())  # nothing lost / reordered / duplicated
        expect_off += m
        idx = co % args.rows
        ok = ok and bool((cv == ref_v[idx]).all())
        both = cv & ref_v[idx]
        ok = ok and bool(np.all(np.abs(cs[both] - ref_s[idx][both]) <= tol))
        checked += m
    return ok and checked == (args.warmup + args.steps) * args.passes * args.rows, checked


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _needs_launch(args) -> bool:
    """``--gpus N > 1`` without a launcher (no ``WORLD_SIZE`` in the environment): this process
    only spawns the N ranks (SURVEY §2.6 F3 — one process per GPU)."""
    return args.gpus > 1 and "WORLD_SIZE" not in os.environ and not os.environ.get("FJA_BENCH_CHILD")


def launch_ranks(args, argv) -> int:
    """Spawn ``--gpus N`` fresh rank processes through ``torch.distributed.run`` and relay rank 0's
    JSON line; returns the launcher's exit status (non-zero if any rank failed — the elastic agent
    then terminates the surviving siblings). Called BEFORE this process makes any GPU call: the
    parent never touches the GPU (no ``torch.cuda.is_available()``), and it never ``exec``s — the
    ranks are children, the parent exits with their status.

    With the RCCL backend every rank needs its own GPU, so N must not exceed the visible device
    count (``torch.cuda.device_count()`` does not initialise the GPU on this image);
    ``FJA_DIST_BACKEND=gloo`` (or ``--rehearse-cpu``) lets N ranks share fewer GPUs / run on CPUs."""
    import signal
    import subprocess

    n = args.gpus
    if not args.rehearse_cpu and os.environ.get("FJA_DIST_BACKEND", "nccl") != "gloo":
        import torch

        have = torch.cuda.device_count()
        if have < n:
            print(json.dumps({"metric": METRIC, "error": f"--gpus {n} but {have} GPU(s) visible "
                              "(set FJA_DIST_BACKEND=gloo to share GPUs between ranks)"}), flush=True)
            return 1
    env = dict(os.environ, FJA_BENCH_CHILD="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or n) // n)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True)
    last_json = None
    try:
        for line in proc.stdout:  # rank 0 is the only rank that prints to stdout
            sys.stdout.write(line)
            sys.stdout.flush()
            if line.lstrip().startswith("{"):
                last_json = line
        rc = proc.wait()
    except BaseException:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=30)
        except Exception:  # noqa: BLE001 - the group is gone or will not die: SIGKILL it
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except OSError:
                pass
        raise
    if rc == 0 and last_json is None:
        print("error: the ranks exited without rank 0's JSON line", file=sys.stderr)
        return 1
    return rc


def main(argv=None) -> int:
    raw_argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(raw_argv)
    if _needs_launch(args):
        return launch_ranks(args, raw_argv)
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

    cpu = bool(args.rehearse_cpu)
    if not cpu and not torch.cuda.is_available():
        print(json.dumps({"metric": METRIC, "error": "no GPU visible"}))
        return 1
    ctx = init_from_env(backend="gloo" if cpu else None, force=args.force_dist)
    device = None if cpu else ctx.device

    def sync():
        if not cpu:
            torch.cuda.synchronize()
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
    doc_paths = [path]
    if args.models > 1:  # --models mode: more distinct documents (seeds) for the model ids to cycle over
        extra = []
        if ctx.rank == 0:
            for k in range(1, max(1, min(args.model_docs, args.models))):
                fd, pk = tempfile.mkstemp(suffix=".pmml", prefix=f"bench-{k}-")
                with os.fdopen(fd, "w") as fh:
                    fh.write(model_text(args, seed=args.seed + k))
                extra.append(pk)
        doc_paths += broadcast_object(extra, ctx)
    t_load = time.perf_counter()
    lm = load_replicated(path, ctx, device, cfg)
    sync()
    load_s = time.perf_counter() - t_load
    model = lm.model
    plan = getattr(model.scorer, "plan", None)

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

    numa_node = None if args.no_numa or cpu else bind_to_gpu_numa(device.index or 0)
    X = torch.from_numpy(stream_matrix(args.rows, args.features, seed=1000 + ctx.rank))
    if not cpu:
        X = X.pin_memory()
    # every distributed run all-gathers (a 1-rank RCCL group under --force-dist takes the same
    # device-mirror / RCCL path as N > 1)
    gather = ctx.is_distributed and not args.no_allgather
    timing = {}

    def barrier_sync():
        sync()
        ctx.barrier()
        sync()

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
        sink = GatherSink(to="all", lockstep=True, keep=cpu) if gather or not ctx.is_distributed else _WaitSink()
        op_cfg = cfg.replace(device_mirror=gather)
        model_ids = None
        if args.models > 1:
            if args.source != "synthetic":
                raise SystemExit("--models needs --source synthetic")
            uuids = [f"00000000-0000-4000-8000-{k:012d}" for k in range(args.models)]
            rng = np.random.default_rng(2000 + ctx.rank)
            codes = torch.from_numpy(rng.integers(0, args.models, args.rows).astype(
                np.uint8 if args.models <= 256 else np.int16))
            if not cpu:
                codes = codes.pin_memory()
            model_ids = (codes, [f"{u}_1" for u in uuids])
        if args.source == "synthetic":
            src = _StepSource(X, args.warmup + args.steps, args.passes, on_step, model_ids)
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
        if args.models > 1:
            from flink_jpmml_amd import AddMessage

            # the control stream (replicated to every rank) registers the models; timestamps order
            # it before the first batch in the deterministic input merge
            adds = [AddMessage(u, 1, doc_paths[k % len(doc_paths)], 0) for k, u in enumerate(uuids)]
            control = env.from_collection(adds, timestamp=lambda m: -1, uid="control")
            stream = env.add_source(src, timestamp=lambda b: b.offset, mode="parallel")
            scored = stream.with_support_stream(control).quick_evaluate(config=op_cfg, uid="serving")
        else:
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
        assert res.records_in == seen + (args.models if args.models > 1 else 0)  # + the AddMessages
        if cpu and gather:
            # rehearsal: every rank checks ITS rows inside every gathered element against its own
            # oracle (row order via the source offsets), then the verdicts are all-gathered
            from flink_jpmml_amd.parallel.dist import all_gather_object

            ok, n_rows = _rehearsal_check(args, sink, ctx, doc_paths)
            job["rehearsal_gather_check"] = all_gather_object(bool(ok), ctx, group=ctx.group("ctrl"))
            job["rehearsal_rows_checked_per_rank"] = all_gather_object(int(n_rows), ctx, group=ctx.group("ctrl"))
            job["rehearsal_rows_gathered_per_rank"] = int(len(sink.scores))
        op = scored.node.factory  # the operator instance this (single-subtask) rank ran
        pipe = getattr(getattr(op, "inner", op), "_pipeline", None)
        if args.models > 1:
            job["models_served"] = len(op.serving_models)
            if ctx.rank == 0 and args.check_rows > 0:  # untimed: every model's rows vs its fp64 oracle
                from flink_jpmml_amd.api.batch import RecordBatch as _RB

                Xc = stream_matrix(args.check_rows, args.features, seed=99, missing_rate=0.02)
                cc = np.random.default_rng(5).integers(0, args.models, args.check_rows)
                pbm = op.score_mixed(_RB(Xc, model_ids=(cc.astype(np.int32), model_ids[1])))
                oracles = [CompiledPmml.from_string(open(pth).read()) for pth in doc_paths]
                errs, vm = [], True
                for k in range(args.models):
                    rows = np.flatnonzero(cc == k)
                    if rows.size == 0:
                        continue
                    sr, vr = oracles[k % len(doc_paths)].score_matrix_oracle(Xc[rows])
                    vm = vm and bool((pbm.valid[rows] == vr).all())
                    both = vr & pbm.valid[rows]
                    if both.any():
                        errs.append(float(np.max(np.abs(pbm.scores[rows][both] - sr[both]))))
                check["mixed_models"] = {"models": args.models, "rows": int(args.check_rows), "valid_match": vm,
                                         "max_abs_err_vs_fp64": max(errs) if errs else None}
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
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if device is not None else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    records_per_s = N * rows_per_step * args.steps / elapsed

    # ---- device-resident kernel throughput (records already in HBM) — reported separately
    n_k = min(args.rows, 1 << 22)
    kernel_ms = float("nan")
    if not cpu:
        kernel_ms = _kernel_ms(plan, X[:n_k], device)

    # ---- p50 latency: one small RecordBatch through model.predict (host records -> host scores)
    from flink_jpmml_amd.api.batch import RecordBatch

    Xl = torch.from_numpy(stream_matrix(args.latency_batch, args.features, seed=7))
    Xl = RecordBatch(Xl if cpu else Xl.pin_memory())
    lats = []
    for i in range(args.latency_iters + 5):
        t1 = time.perf_counter()
        model.predict(Xl).wait()
        if i >= 5:
            lats.append((time.perf_counter() - t1) * 1e3)
    p50 = float(np.percentile(lats, 50))
    p99 = float(np.percentile(lats, 99))

    if ctx.rank == 0:
        default = args.model == "gbdt" and args.source == "synthetic" and args.models == 1
        metric = METRIC if default else f"records/sec (whole node) on {MODELS[args.model][1]} PMML; p50 latency"
        if args.models > 1:
            metric = (f"records/sec (whole node), dynamic serving of {args.models} x {args.trees}-tree "
                      f"{MODELS[args.model][1]} PMML models, every record names a random model")
        if args.source != "synthetic":
            metric += f" [source: {args.source} record file, end to end incl. ingest]"
        if cpu:
            metric = "[CPU REHEARSAL, not a benchmark] " + metric
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
                "models": args.models,
                "model_docs": len(doc_paths),
            },
            "p50_latency_ms": p50,
            "p99_latency_ms": p99,
            "latency_batch_rows": args.latency_batch,
            "kernel_only_records_per_s_per_gpu": None if cpu else n_k / (kernel_ms / 1e3),
            "kernel_ms_per_1M_rows": None if cpu else kernel_ms * (1 << 20) / n_k,
            "h2d_gbps_effective": rows_per_step * args.features * 4 * args.steps / elapsed / 1e9,
            "job": job,
            "model_load_broadcast_s": load_s,
            "timed_region_s": elapsed,
            "plan": {"layout": getattr(plan, "layout", None), "depth": getattr(plan, "depth", None),
                     "chunk_trees": getattr(plan, "chunk_trees", None), "kind": getattr(plan, "kind", None)},
            "check": check,
            "rehearsal_cpu": cpu,
            "metrics": {k: v for k, v in METRICS.summary()["counters"].items() if not k.startswith("model_cache")},
        }
        print(json.dumps(out), flush=True)
        for pth in doc_paths:
            try:
                os.unlink(pth)
            except OSError:
                pass
    if ctx.is_distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
