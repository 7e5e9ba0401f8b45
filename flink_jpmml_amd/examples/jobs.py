"""Example jobs — the reference's `E/*.scala` applications as CLI commands.

    python -m flink_jpmml_amd.examples quick     --model kmeans.xml --output out.txt [--device cuda]
    python -m flink_jpmml_amd.examples evaluate  --model kmeans.xml --output out.txt
    python -m flink_jpmml_amd.examples dynamic   --models a.xml,b.xml --output out.txt --gen-policy finite \
                                                 --intervalCheckpoint 1000 --maxIntervalControlStream 0
    python -m flink_jpmml_amd.examples checkpoint --output out.txt --control-file paths.txt

Flags keep the reference's names (`E/util/DynamicParams.scala:28-68`,
`E/util/EnsureParameters.scala:24-29`); ``--device``/``--batch-size`` switch to micro-batched GPU
scoring. ``--intervalCheckpoint`` counts records (the runtime's barriers are count based).

Scoring configuration (:class:`~flink_jpmml_amd.config.ScoringConfig`) from flags:
``--max-batch-latency-ms`` (size-or-time flush), ``--precision fp32|bf16|fp8``, ``--fallback
host|warn|error``, ``--cache-capacity``, ``--micro-batch``, ``--watchdog-s``; ``--rate`` limits the
Iris source to N records/s (the reference's sources emit 1 record/s, `E/sources/IrisSource.scala:52`);
``--metrics-out PATH`` writes the run's counters / latency histograms as JSON.
"""

from __future__ import annotations

import argparse
import socket
import sys
import uuid
from typing import List, Optional

from ..api.reader import ModelReader
from ..config import ScoringConfig
from ..domain.control import AddMessage
from ..stream.datastream import StreamExecutionEnvironment
from ..utils.metrics import METRICS
from .sources import ControlSource, IrisSource, ids_and_paths, now_ms


def _write(out: List, path: Optional[str]) -> None:
    if path in (None, "-"):
        for x in out:
            print(x)
        return
    with open(path, "w") as fh:
        for x in out:
            fh.write(f"{x}\n")


def scoring_config(args) -> ScoringConfig:
    """The job's :class:`ScoringConfig` from its CLI flags (unset flags keep the defaults)."""
    kw = dict(batch_size=args.batch_size, device=args.device, max_batch_latency_ms=args.max_batch_latency_ms,
              precision=args.precision, fallback=args.fallback, cache_capacity=args.cache_capacity,
              micro_batch=args.micro_batch, watchdog_s=args.watchdog_s)
    return ScoringConfig(**{k: v for k, v in kw.items() if v is not None})


def _env(args) -> StreamExecutionEnvironment:
    return StreamExecutionEnvironment(args.parallelism, config=scoring_config(args))


def quick_evaluate_kmeans(args) -> List:
    """X1 (`E/QuickEvaluateKmeans.scala:29-54`): Iris vectors → quick_evaluate → sink."""
    env = _env(args)
    vectors = env.add_source(IrisSource(None, n=args.records, rate=args.rate, seed=args.seed)).map(
        lambda e: e.to_vector())
    out = vectors.quick_evaluate(ModelReader(args.model), batch_size=args.batch_size, device=args.device).collect()
    _write(out, args.output)
    return out


def evaluate_kmeans(args) -> List:
    """X2 (`E/EvaluateKmeans.scala:29-57`): full UDF with ``predict(vec, Some(0.0))``."""
    env = _env(args)
    events = env.add_source(IrisSource(None, n=args.records, rate=args.rate, seed=args.seed))

    def udf(event, model):
        prediction = model.predict(event.to_vector(), 0.0)
        return event, prediction.value.get_or_else(-1.0)

    out = events.evaluate(ModelReader(args.model), udf, batch_size=args.batch_size, device=args.device).collect()
    _write(out, args.output)
    return out


def dynamic_evaluate_kmeans(args) -> List:
    """X3 (`E/DynamicEvaluateKmeans.scala:38-67`): events tagged with model ids + a control stream."""
    paths = [p for p in args.models.split(",") if p]
    idp = ids_and_paths(paths)
    env = _env(args)
    if args.intervalCheckpoint:
        env.enable_checkpointing(args.intervalCheckpoint, args.checkpoint_dir)
    control = env.add_source(ControlSource(idp, args.gen_policy, n=args.control_messages,
                                           max_interval_ms=args.maxIntervalControlStream, seed=args.seed),
                             timestamp=lambda m: m.occurred_on)
    events = env.add_source(IrisSource(list(idp), n=args.records, rate=args.rate, seed=args.seed),
                            timestamp=lambda e: e.occurred_on)

    def udf(event, model):
        return event.model_id, model.predict(event.to_vector(), None)

    out = events.with_support_stream(control).evaluate(udf, batch_size=args.batch_size, device=args.device,
                                                       uid="dynamic-kmeans").collect(restore=args.restore)
    _write(out, args.output)
    return out


def _control_lines(args):
    if args.control_file:
        with open(args.control_file) as fh:
            for line in fh:
                line = line.strip()
                if line:
                    yield line
    elif args.socket:
        host, port = args.socket.split(":")
        with socket.create_connection((host, int(port))) as s, s.makefile() as fh:
            for line in fh:
                line = line.strip()
                if line:
                    yield line


def checkpoint_evaluate(args) -> List:
    """X4 (`E/CheckpointEvaluate.scala:36-102`): fixed ids, each control line is a model path mapped
    to ``AddMessage(randomId, 1, path, now)``; metadata checkpoints every N records."""
    ids = [str(uuid.UUID(int=1)), str(uuid.UUID(int=2))]
    env = _env(args)
    env.enable_checkpointing(args.intervalCheckpoint or 10, args.checkpoint_dir)
    lines = list(_control_lines(args))
    ctrl = [AddMessage(ids[i % len(ids)], 1, p, now_ms()) for i, p in enumerate(lines)]
    control = env.from_collection(ctrl, timestamp=lambda m: m.occurred_on)
    events = env.add_source(IrisSource(ids, n=args.records, rate=args.rate, seed=args.seed),
                            timestamp=lambda e: e.occurred_on)
    out = events.with_support_stream(control).evaluate(
        lambda e, m: (e.model_id, m.predict(e.to_vector()).value.get_or_else(-1.0)),
        uid="checkpoint-evaluate").collect(restore=args.restore)
    _write(out, args.output)
    return out


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m flink_jpmml_amd.examples")
    sub = p.add_subparsers(dest="cmd", required=True)

    def common(sp):
        sp.add_argument("--output", required=True)
        sp.add_argument("--records", type=int, default=100)
        sp.add_argument("--parallelism", type=int, default=1)
        sp.add_argument("--batch-size", type=int, default=None)
        sp.add_argument("--device", default=None)
        sp.add_argument("--seed", type=int, default=0)
        sp.add_argument("--rate", type=float, default=None, help="source records per second (None: unthrottled)")
        sp.add_argument("--max-batch-latency-ms", type=float, default=None)
        sp.add_argument("--precision", default=None, choices=("fp32", "bf16", "fp8"))
        sp.add_argument("--fallback", default=None, choices=("host", "warn", "error"))
        sp.add_argument("--cache-capacity", type=int, default=None)
        sp.add_argument("--micro-batch", type=int, default=None)
        sp.add_argument("--watchdog-s", type=float, default=None)
        sp.add_argument("--metrics-out", default=None, help="write the run's metrics summary (JSON) here")

    for name, fn in (("quick", quick_evaluate_kmeans), ("evaluate", evaluate_kmeans)):
        sp = sub.add_parser(name)
        sp.add_argument("--model", required=True)
        common(sp)
        sp.set_defaults(fn=fn)
    sp = sub.add_parser("dynamic")
    sp.add_argument("--models", required=True, help="comma-separated model paths")
    sp.add_argument("--gen-policy", default="random", choices=ControlSource.POLICIES)
    sp.add_argument("--intervalCheckpoint", type=int, default=1000)
    sp.add_argument("--maxIntervalControlStream", type=int, default=0)
    sp.add_argument("--control-messages", type=int, default=None)
    sp.add_argument("--checkpoint-dir", default=None)
    sp.add_argument("--restore", default=None)
    common(sp)
    sp.set_defaults(fn=dynamic_evaluate_kmeans)
    sp = sub.add_parser("checkpoint")
    sp.add_argument("--control-file", default=None)
    sp.add_argument("--socket", default=None, help="host:port, one model path per line")
    sp.add_argument("--intervalCheckpoint", type=int, default=10)
    sp.add_argument("--checkpoint-dir", default=None)
    sp.add_argument("--restore", default=None)
    common(sp)
    sp.set_defaults(fn=checkpoint_evaluate)
    return p


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    if getattr(args, "cmd", None) == "dynamic" and args.gen_policy != "finite" and args.control_messages is None:
        args.control_messages = 10  # bounded by default so the example terminates
    METRICS.reset()
    args.fn(args)
    if args.metrics_out:
        METRICS.dump(args.metrics_out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
