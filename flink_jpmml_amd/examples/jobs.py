"""Example jobs — the reference's `E/*.scala` applications as CLI commands.

    python -m flink_jpmml_amd.examples quick     --model kmeans.xml --output out.txt [--device cuda]
    python -m flink_jpmml_amd.examples evaluate  --model kmeans.xml --output out.txt
    python -m flink_jpmml_amd.examples dynamic   --models a.xml,b.xml --output out.txt --gen-policy random \
                                                 --intervalCheckpoint 1000 --maxIntervalControlStream 5000
    python -m flink_jpmml_amd.examples checkpoint --output out.txt --socket localhost:9999   # nc -lk 9999

Flags keep the reference's names and defaults (`E/util/DynamicParams.scala:28-68`,
`E/util/EnsureParameters.scala:24-29`): ``--intervalCheckpoint`` is a time interval in ms,
``--maxIntervalControlStream`` 5000 ms, events at 1 record/s (``--rate``); every job streams its
output with ``writeAsText`` semantics. ``--device``/``--batch-size`` switch to micro-batched GPU
scoring.

Scoring configuration (:class:`~flink_jpmml_amd.config.ScoringConfig`) from flags:
``--max-batch-latency-ms`` (size-or-time flush), ``--precision fp32|bf16|fp8``, ``--fallback
host|warn|error``, ``--cache-capacity``, ``--micro-batch``, ``--watchdog-s``; ``--rate`` limits the
Iris source to N records/s (the reference's sources emit 1 record/s, `E/sources/IrisSource.scala:52`);
``--metrics-out PATH`` writes the run's counters / latency histograms as JSON.
"""

from __future__ import annotations

import argparse
import sys
from typing import List, Optional

from ..api.reader import ModelReader
from ..config import ScoringConfig
from ..domain.control import AddMessage
from ..stream.datastream import StreamExecutionEnvironment
from ..utils.metrics import METRICS
from .sources import ControlSource, IrisSource, ids_and_paths, now_ms


def _sink(stream, args, keep: bool = True) -> List:
    """``writeAsText(output)`` — lines are written as results arrive (the file grows while the
    job runs) — plus an in-memory copy the CLI returns (bounded runs only)."""
    out: List = []
    stream.write_as_text(args.output)
    if keep:
        stream.add_sink(out.append)
    return out


def scoring_config(args) -> ScoringConfig:
    """The job's :class:`ScoringConfig` from its CLI flags (unset flags keep the defaults)."""
    kw = dict(batch_size=args.batch_size, device=args.device, max_batch_latency_ms=args.max_batch_latency_ms,
              precision=args.precision, fallback=args.fallback, cache_capacity=args.cache_capacity,
              micro_batch=args.micro_batch, watchdog_s=args.watchdog_s)
    return ScoringConfig(**{k: v for k, v in kw.items() if v is not None})


def _env(args) -> StreamExecutionEnvironment:
    return StreamExecutionEnvironment(args.parallelism, config=scoring_config(args))


def _records(args) -> Optional[int]:
    """``--records``: ``None`` (unbounded, the reference's default) for 0 or less."""
    return args.records if args.records and args.records > 0 else None


def _rate(args) -> Optional[float]:
    return args.rate if args.rate and args.rate > 0 else None


def quick_evaluate_kmeans(args) -> List:
    """X1 (`E/QuickEvaluateKmeans.scala:29-54`): Iris vectors → quick_evaluate → writeAsText."""
    env = _env(args)
    vectors = env.add_source(IrisSource(None, n=_records(args), rate=_rate(args), seed=args.seed)).map(
        lambda e: e.to_vector())
    out = _sink(vectors.quick_evaluate(ModelReader(args.model), batch_size=args.batch_size, device=args.device), args,
                keep=_records(args) is not None)
    env.execute("Quick Evaluate Kmeans")
    return out


def evaluate_kmeans(args) -> List:
    """X2 (`E/EvaluateKmeans.scala:29-57`): full UDF with ``predict(vec, Some(0.0))``."""
    env = _env(args)
    events = env.add_source(IrisSource(None, n=_records(args), rate=_rate(args), seed=args.seed))

    def udf(event, model):
        prediction = model.predict(event.to_vector(), 0.0)
        return event, prediction.value.get_or_else(-1.0)

    out = _sink(events.evaluate(ModelReader(args.model), udf, batch_size=args.batch_size, device=args.device), args,
                keep=_records(args) is not None)
    env.execute("Evaluate Kmeans")
    return out


def _enable_checkpointing(env: StreamExecutionEnvironment, args) -> None:
    """``env.enableCheckpointing(ckpInterval, EXACTLY_ONCE)``: ``--intervalCheckpoint`` is in ms,
    like the reference's (`E/util/DynamicParams.scala:38`)."""
    if args.intervalCheckpoint and args.intervalCheckpoint > 0:
        env.enable_checkpointing(interval_ms=args.intervalCheckpoint, directory=args.checkpoint_dir)


def _predict_udf(event, model):
    """The reference's UDF (`E/DynamicEvaluateKmeans.scala:54-60`, `E/CheckpointEvaluate.scala:89-95`):
    ``(event, model.predict(vectorized, Some(0.0)).value)``."""
    return event, model.predict(event.to_vector(), 0.0).value


def dynamic_evaluate_kmeans(args) -> List:
    """X3 (`E/DynamicEvaluateKmeans.scala:38-67`): events tagged with model ids + a control stream
    with random gaps up to ``--maxIntervalControlStream`` ms; events keep flowing meanwhile."""
    paths = [p for p in args.models.split(",") if p]
    idp = ids_and_paths(paths)
    env = _env(args)
    _enable_checkpointing(env, args)
    control = env.add_source(ControlSource(idp, args.gen_policy, n=args.control_messages,
                                           max_interval_ms=args.maxIntervalControlStream, seed=args.seed))
    events = env.add_source(IrisSource(list(idp), n=_records(args), rate=_rate(args), seed=args.seed))
    preds = events.with_support_stream(control).evaluate(_predict_udf, batch_size=args.batch_size,
                                                         device=args.device, uid="dynamic-kmeans")
    out = _sink(preds, args, keep=_records(args) is not None)
    env.execute("Dynamic Clustering Example", restore=args.restore)
    return out


def checkpoint_evaluate(args) -> List:
    """X4 (`E/CheckpointEvaluate.scala:36-102`): two fixed ids; 1 Hz Iris events; the control
    stream is a **live socket** (``--socket host:port``, one model path per line, mapped to
    ``AddMessage(randomId, 1, path, now)``) or a file; time-based EXACTLY_ONCE checkpoints; the
    output file is written as results arrive."""
    import random

    ids = ["4897c9f4-5226-43c7-8f2d-f9fd388cf2bc", "5f919c52-2ef8-4ff2-94b2-2e64bb85005e"]
    rng = random.Random(args.seed)
    env = _env(args)
    _enable_checkpointing(env, args)
    if args.socket:
        host, port = args.socket.rsplit(":", 1)
        lines = env.socket_text_stream(host, int(port), uid="control-socket")
    elif args.control_file:
        with open(args.control_file) as fh:
            lines = env.from_collection([ln.strip() for ln in fh if ln.strip()], uid="control-file")
    else:
        raise SystemExit("checkpoint: give --socket host:port or --control-file")
    control = lines.filter(lambda ln: bool(ln.strip())).map(
        lambda path: AddMessage(ids[rng.randrange(len(ids))], 1, path.strip(), now_ms()))
    events = env.add_source(IrisSource(ids, n=_records(args), rate=_rate(args), seed=args.seed))
    preds = events.with_support_stream(control).evaluate(_predict_udf, batch_size=args.batch_size,
                                                         device=args.device, uid="checkpoint-evaluate")
    out = _sink(preds, args, keep=_records(args) is not None)
    env.execute("Checkpoint Evaluate Example", restore=args.restore)
    return out


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m flink_jpmml_amd.examples")
    sub = p.add_subparsers(dest="cmd", required=True)

    def common(sp):
        sp.add_argument("--output", required=True)
        sp.add_argument("--records", type=int, default=0,
                        help="Iris records to emit; 0 (default) = unbounded, the job runs until cancelled like "
                             "the reference's (IrisSource.scala:52)")
        sp.add_argument("--parallelism", type=int, default=1)
        sp.add_argument("--batch-size", type=int, default=None)
        sp.add_argument("--device", default="auto", help="auto (GPU when visible, default), cuda[:i] or cpu")
        sp.add_argument("--seed", type=int, default=0)
        sp.add_argument("--rate", type=float, default=1.0,
                        help="Iris records per second (reference: 1, IrisSource.scala:52); 0 = unthrottled")
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
    sp.add_argument("--intervalCheckpoint", type=int, default=1000, help="checkpoint interval in ms (0 = off)")
    sp.add_argument("--maxIntervalControlStream", type=int, default=5000,
                    help="max random gap between control messages, ms (reference default 5000)")
    sp.add_argument("--control-messages", type=int, default=None,
                    help="control messages to emit (default: unbounded; 10 when --records bounds the run)")
    sp.add_argument("--checkpoint-dir", default=None)
    sp.add_argument("--restore", default=None)
    common(sp)
    sp.set_defaults(fn=dynamic_evaluate_kmeans)
    sp = sub.add_parser("checkpoint")
    sp.add_argument("--control-file", default=None)
    sp.add_argument("--socket", default=None, help="host:port, one model path per line")
    sp.add_argument("--intervalCheckpoint", type=int, default=1000, help="checkpoint interval in ms (0 = off)")
    sp.add_argument("--checkpoint-dir", default=None)
    sp.add_argument("--restore", default=None)
    common(sp)
    sp.set_defaults(fn=checkpoint_evaluate)
    return p


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    if getattr(args, "cmd", None) == "dynamic" and args.gen_policy != "finite" and args.control_messages is None \
            and _records(args) is not None:
        # a bounded run (--records N) ends with its events: bound the loop / random control stream
        # too. The default (unbounded events and control) runs until cancelled, like the reference.
        args.control_messages = 10
    METRICS.reset()
    args.fn(args)
    if args.metrics_out:
        METRICS.dump(args.metrics_out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
