"""``StreamExecutionEnvironment`` / ``DataStream`` / ``ConnectedStreams`` + the scoring DSL.

DSL (reference `S/package.scala:58-143`)::

    env = StreamExecutionEnvironment.get_execution_environment()   # under torchrun: one rank per GPU
    out = env.from_collection(events).evaluate(ModelReader(path), lambda e, m: m.predict(e.vec))
    out = vectors.quick_evaluate(ModelReader(path))                       # -> (Prediction, vector)
    out = events.with_support_stream(control).evaluate(lambda e, m: ...)  # dynamic serving
    results = out.collect()                                               # runs the job

Columnar fast path (the MI355X way to feed a GPU)::

    batches = env.from_batches(X_pinned, batch_rows=1 << 22)      # RecordBatch elements
    scored = batches.quick_evaluate(ModelReader(path), config=ScoringConfig(device="cuda"))
    # -> (PredictionBatch, RecordBatch) per batch; PredictionBatch[i] == model.predict(row i)

Every scoring entry point accepts ``config=`` (:class:`~flink_jpmml_amd.config.ScoringConfig`:
batch size, latency bound, device, precision, fallback policy, …) and the legacy shortcuts
``batch_size=`` / ``device=``. Under ``torchrun`` :meth:`StreamExecutionEnvironment.get_execution_environment`
joins the process group and every operator runs as one subtask per rank (SURVEY §2.7 DP).
"""

from __future__ import annotations

import json
import os
from typing import Any, Callable, Iterable, List, Optional, Sequence, Tuple

from ..api.reader import ModelReader
from ..config import ScoringConfig
from .clock import Clock
from .functions import CoProcessFunction, SinkFunction, SourceFunction
from .operators import EvaluationCoFunction, EvaluationFunction, QuickEvaluationFunction
from .runtime import Executor, JobExecutionResult, Node, SimulatedFailure
from .sources import BatchSource, CollectionSource, ReplicatedSource, SocketTextSource, TextBatchSource
from .state import CheckpointStorage

_DIST: dict = {}  # the process's DistContext (process groups are created once per process)


def _uid(env: "StreamExecutionEnvironment", prefix: str) -> str:
    """Per-environment sequential ids: the same job code builds the same ids in every run and on
    every rank, so checkpoint manifests (operator state, source offsets) map back on restore."""
    env._uid_counter += 1
    return f"{prefix}-{env._uid_counter}"


class CollectSink(SinkFunction):
    """Collects into a shared list (the reference's test sink, `T/utils/FlinkTestKits.scala:58-62`).
    Under data parallelism :meth:`DataStream.collect` gathers every rank's list (rank order)."""

    def __init__(self, target: Optional[list] = None):
        self.values = target if target is not None else []

    def invoke(self, value: Any) -> None:
        self.values.append(value)

    def invoke_many(self, values: list) -> None:
        self.values.extend(values)

    def __getstate__(self):
        return self.__dict__  # keeps the shared list when cloned for parallel subtasks


class FileSink(SinkFunction):
    """Exactly-once text sink: one JSON line per element, two-phase committed per checkpoint.

    Elements go to an in-progress buffer; ``pre_commit(cid)`` writes them to
    ``<dir>/part-<rank>-<cid>.pending``; ``commit(cid)`` renames it to ``.jsonl`` once the
    checkpoint manifest is durable (end of input commits the rest as ``part-<rank>-final``).
    ``recover(cid)`` (called on restore from checkpoint ``cid``) finishes the crashed run's
    transactions like Flink's two-phase-commit sink: parts pre-committed for checkpoints
    ``<= cid`` are covered by the restored manifest and are committed (the process may have died
    between writing the manifest and renaming them); newer pending parts are discarded (the
    restored job re-produces them). The committed parts of both runs together equal one
    uninterrupted run — no duplicates, no gaps."""

    def __init__(self, directory: str, encode: Optional[Callable[[Any], Any]] = None):
        self.directory = directory
        self.encode = encode or _json_default
        self._buf: List[str] = []
        self._pending: List[Tuple[int, str]] = []
        self.rank = 0

    def open(self, context=None) -> None:  # noqa: A003
        os.makedirs(self.directory, exist_ok=True)
        if context is not None:
            self.rank = context.index_of_this_subtask

    def invoke(self, value: Any) -> None:
        self._buf.append(json.dumps(self.encode(value), default=_json_default))

    def _name(self, cid: int) -> str:
        tag = "final" if cid < 0 else f"{cid:06d}"
        return os.path.join(self.directory, f"part-{self.rank:03d}-{tag}")

    def pre_commit(self, cid: int) -> None:
        path = self._name(cid) + ".pending"
        with open(path, "w") as fh:
            fh.write("".join(x + "\n" for x in self._buf))
            fh.flush()
            os.fsync(fh.fileno())
        self._buf = []
        self._pending.append((cid, path))

    def commit(self, cid: int) -> None:
        keep = []
        for c, path in self._pending:
            if c == cid or cid < 0:
                os.replace(path, path[: -len(".pending")] + ".jsonl")
            else:
                keep.append((c, path))
        self._pending = keep

    def recover(self, restored_cid: Optional[int] = None) -> None:
        prefix = f"part-{self.rank:03d}-"
        for f in sorted(os.listdir(self.directory)):
            if not (f.startswith(prefix) and f.endswith(".pending")):
                continue
            path = os.path.join(self.directory, f)
            tag = f[len(prefix): -len(".pending")]
            if tag.isdigit() and restored_cid is not None and int(tag) <= int(restored_cid):
                os.replace(path, path[: -len(".pending")] + ".jsonl")
            else:
                os.remove(path)

    @staticmethod
    def read(directory: str) -> List[Any]:
        """Committed output in (rank, checkpoint) order."""
        out = []
        for f in sorted(os.listdir(directory)):
            if f.endswith(".jsonl"):
                with open(os.path.join(directory, f)) as fh:
                    out.extend(json.loads(line) for line in fh if line.strip())
        return out


class TextSink(SinkFunction):
    """``writeAsText(path)`` (`E/EvaluateKmeans.scala:53`, `E/CheckpointEvaluate.scala:97-98`):
    one line per element, written and flushed **as results arrive** (the file grows while the job
    runs; at-least-once across restarts, like Flink's ``writeAsText``). Under data parallelism
    rank ``r`` writes ``<path>.<r>`` unless ``path`` is ``"-"`` (stdout)."""

    def __init__(self, path: str, fmt: Optional[Callable[[Any], str]] = None, flush_every: int = 1):
        self.path = path
        self.fmt = fmt or str
        self.flush_every = max(1, int(flush_every))
        self._fh = None
        self._n = 0

    def open(self, context=None) -> None:  # noqa: A003
        import sys

        if self.path in (None, "-"):
            self._fh = sys.stdout
            return
        path = self.path
        if context is not None and context.number_of_parallel_subtasks > 1:
            path = f"{path}.{context.index_of_this_subtask}"
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._fh = open(path, "w")

    def invoke(self, value: Any) -> None:
        self._fh.write(self.fmt(value) + "\n")
        self._n += 1
        if self._n % self.flush_every == 0:
            self._fh.flush()

    def close(self) -> None:
        import sys

        if self._fh is not None:
            self._fh.flush()
            if self._fh is not sys.stdout:
                self._fh.close()
            self._fh = None

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_fh"] = None
        return d


def _json_default(x: Any) -> Any:
    from ..api.batch import PredictionBatch
    from ..domain.prediction import Prediction

    if isinstance(x, Prediction):
        return None if x.value.is_empty else x.value.get()
    if isinstance(x, PredictionBatch):
        return [None if not v else float(s) for s, v in zip(x.scores, x.valid)]
    if isinstance(x, (tuple, list)):
        return [_json_default(y) for y in x]
    if hasattr(x, "tolist"):
        return x.tolist()
    if hasattr(x, "__dict__"):
        return {k: _json_default(v) for k, v in vars(x).items()}
    return x if isinstance(x, (int, float, str, bool, type(None), dict)) else repr(x)


class _FnSink(SinkFunction):
    def __init__(self, fn: Callable[[Any], None]):
        self.fn = fn

    def invoke(self, value: Any) -> None:
        self.fn(value)

    def invoke_many(self, values: list) -> None:
        fn = self.fn
        for v in values:
            fn(v)


class StreamExecutionEnvironment:
    def __init__(self, parallelism: int = 1, config: Optional[ScoringConfig] = None, dist_ctx=None,
                 clock: Optional[Clock] = None):
        self.parallelism = parallelism
        self.config = config
        self.dist_ctx = dist_ctx
        self.clock = clock
        self.checkpoint_every: Optional[int] = None
        self.checkpoint_interval_ms: Optional[float] = None
        self.input_mode = "auto"
        self.gc_tuning = True
        self.checkpoint_storage = CheckpointStorage()
        self.fail_after: Optional[int] = None
        self.copy_operators = False
        self._sinks: List[Node] = []
        self._uid_counter = 0
        if dist_ctx is not None and dist_ctx.is_distributed:
            self.parallelism = dist_ctx.world_size

    @staticmethod
    def get_execution_environment(config: Optional[ScoringConfig] = None, backend: Optional[str] = None,
                                  force_distributed: bool = False) -> "StreamExecutionEnvironment":
        """Under ``torchrun`` (``WORLD_SIZE > 1``): join the process group (RCCL on GPUs, gloo on
        CPUs) and return an environment whose operators run one subtask per rank. Otherwise a
        local environment. ``force_distributed`` forms a 1-rank group (RCCL on one GPU)."""
        ctx = None
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 or force_distributed:
            ctx = _DIST.get("ctx")
            if ctx is None:
                from ..parallel.dist import init_from_env

                ctx = _DIST["ctx"] = init_from_env(backend=backend, force=force_distributed)
        return StreamExecutionEnvironment(config=config, dist_ctx=ctx)

    getExecutionEnvironment = get_execution_environment  # noqa: N815

    @property
    def is_distributed(self) -> bool:
        return self.dist_ctx is not None and self.dist_ctx.is_distributed

    def set_parallelism(self, p: int) -> "StreamExecutionEnvironment":
        if self.is_distributed and int(p) != self.dist_ctx.world_size:
            raise ValueError(f"under torchrun the parallelism is the world size ({self.dist_ctx.world_size})")
        self.parallelism = int(p)
        return self

    setParallelism = set_parallelism  # noqa: N815

    def set_config(self, config: ScoringConfig) -> "StreamExecutionEnvironment":
        """Job-wide scoring defaults (operators without an explicit ``config=`` use them)."""
        self.config = config
        return self

    def set_clock(self, clock: Clock) -> "StreamExecutionEnvironment":
        """Processing-time clock (tests inject a :class:`~flink_jpmml_amd.stream.clock.ManualClock`)."""
        self.clock = clock
        return self

    def enable_checkpointing(self, interval_ms: Optional[float] = None, directory: Optional[str] = None,
                             every_n_records: Optional[int] = None) -> "StreamExecutionEnvironment":
        """``enableCheckpointing(interval)`` (`E/DynamicEvaluateKmeans.scala:48`): a checkpoint
        every ``interval_ms`` of processing time — across ranks rank 0 decides and every rank
        snapshots at its own exact cut. ``every_n_records`` instead places count-based barriers on
        the primary source's global offset (deterministic: aligned across ranks without
        communication; for replayable inputs and tests)."""
        if (interval_ms is None) == (every_n_records is None):
            raise ValueError("give exactly one of interval_ms / every_n_records")
        if every_n_records is not None:
            self.checkpoint_every, self.checkpoint_interval_ms = int(every_n_records), None
        else:
            if float(interval_ms) <= 0:
                raise ValueError("interval_ms must be > 0")
            self.checkpoint_every, self.checkpoint_interval_ms = None, float(interval_ms)
        if directory is not None:
            self.checkpoint_storage = CheckpointStorage(directory)
        elif self.config is not None and self.config.checkpoint_dir:
            self.checkpoint_storage = CheckpointStorage(self.config.checkpoint_dir)
        elif os.environ.get("FJA_CHECKPOINT_DIR"):  # set by the restart supervisor
            self.checkpoint_storage = CheckpointStorage(os.environ["FJA_CHECKPOINT_DIR"])
        return self

    enableCheckpointing = enable_checkpointing  # noqa: N815

    def set_input_mode(self, mode: str) -> "StreamExecutionEnvironment":
        """``auto`` (default: live reader threads when any source can block, else the
        deterministic merge), ``live`` or ``deterministic`` (see :mod:`~flink_jpmml_amd.stream.inputs`)."""
        if mode not in ("auto", "live", "deterministic"):
            raise ValueError(f"input mode must be auto / live / deterministic, not {mode!r}")
        self.input_mode = mode
        return self

    def inject_failure(self, after_records: Optional[int]) -> "StreamExecutionEnvironment":
        """Fault injection: fail the job once ``after_records`` source records were processed."""
        self.fail_after = after_records
        return self

    # ------------------------------------------------------------------ sources
    def _source(self, src: Any, name: str, timestamp=None, mode: str = "shard") -> "DataStream":
        node = Node("source", name, 1, source=src, timestamp_fn=timestamp, uid=_uid(self, "src"), dist_mode=mode)
        return DataStream(self, node)

    def from_collection(self, items: Iterable[Any], timestamp: Optional[Callable[[Any], Any]] = None,
                        name: str = "collection", uid: Optional[str] = None) -> "DataStream":
        s = self._source(CollectionSource(items), name, timestamp)
        if uid:
            s.node.uid = uid
        return s

    fromCollection = from_collection  # noqa: N815

    def from_elements(self, *items: Any) -> "DataStream":
        return self.from_collection(items)

    def add_source(self, source: SourceFunction, timestamp: Optional[Callable[[Any], Any]] = None,
                   name: str = "source", mode: Optional[str] = None, uid: Optional[str] = None) -> "DataStream":
        """``mode`` under torchrun: ``shard`` (default for replayable sources), ``parallel`` (every
        rank runs its own instance; default for sources with ``open_subtask``), ``replicate``
        (every rank reads it all) or ``leader`` (rank 0 reads, elements are broadcast)."""
        if mode is None:
            mode = "parallel" if hasattr(source, "open_subtask") else "shard"
        if mode == "leader":  # rank 0 reads; elements are sharded, or replicated behind broadcast()
            source, mode = ReplicatedSource(source, self.dist_ctx), "shard"
        s = self._source(source, name, timestamp, mode)
        if uid:
            s.node.uid = uid
        return s

    addSource = add_source  # noqa: N815

    def from_batches(self, data: Any, batch_rows: Optional[int] = None, repeat: int = 1,
                     model_id: Optional[str] = None, mode: str = "shard", name: str = "batches",
                     uid: Optional[str] = None) -> "DataStream":
        """Columnar source of RecordBatch elements from a ``[rows, F]`` matrix (cut into
        ``batch_rows``) or an iterable of matrices / RecordBatches."""
        s = self._source(BatchSource(data, batch_rows, repeat, model_id), name, None, mode)
        if uid:
            s.node.uid = uid
        return s

    fromBatches = from_batches  # noqa: N815

    def read_text_batches(self, path: str, model: Any, batch_rows: int = 1 << 16, **kw) -> "DataStream":
        """Delimited text file → RecordBatches via the native C++ ingest (pinned output). Under
        torchrun every rank parses only its own byte range (rank-local split, F3)."""
        return self._source(TextBatchSource(path, model, batch_rows, **kw), "text-batches", None, "parallel")

    def read_binary_batches(self, path: str, batch_rows: int = 1 << 20, threads: int = 4, repeat: int = 1,
                            model_id: Optional[str] = None) -> "DataStream":
        """Binary fp32 record file (:mod:`~flink_jpmml_amd.stream.binary`) → pinned RecordBatches:
        memory-mapped, copied into pinned buffers by ``threads`` workers, no parsing. Under torchrun
        every rank maps only its own row range."""
        from .binary import BinaryBatchSource

        return self._source(BinaryBatchSource(path, batch_rows, threads, repeat=repeat, model_id=model_id),
                            "binary-batches", None, "parallel")

    def socket_binary_stream(self, host: str, port: int, model_id: Optional[str] = None) -> "DataStream":
        """TCP stream of binary record frames (``binary.send_binary``) → pinned RecordBatches."""
        from .binary import SocketBinarySource

        return self._source(SocketBinarySource(host, port, model_id=model_id), "binary-socket", None, "parallel")

    def socket_text_stream(self, host: str, port: int, delimiter: str = "\n", max_retry: int = 0,
                           uid: Optional[str] = None) -> "DataStream":
        """``socketTextStream(host, port)`` (`E/CheckpointEvaluate.scala:80-82`): lines read live
        as they arrive. Under torchrun rank 0 reads and the lines are replicated (behind
        ``broadcast()`` / ``with_support_stream``) or sharded across ranks."""
        s = self.add_source(SocketTextSource(host, port, delimiter, max_retry), name="socket", mode="leader")
        if uid:
            s.node.uid = uid
        return s

    socketTextStream = socket_text_stream  # noqa: N815

    def from_either(self, sequence: Sequence[Tuple[str, Any]], uid: Optional[str] = None
                    ) -> Tuple["DataStream", "DataStream"]:
        """One ordered source split into a left and a right stream: ``[("L", ev), ("R", ctrl)]``.
        The runtime delivers the elements in exactly this order (deterministic two-input tests,
        the analogue of `T/utils/FlinkTestKits.scala:44-55`). Under torchrun ``L`` elements are
        sharded across ranks and ``R`` elements replicated to every rank."""
        tagged = self._source(CollectionSource(list(sequence)), "either", None, "either")
        if uid:
            tagged.node.uid = uid
        left = tagged.filter(lambda t: t[0] == "L").map(lambda t: t[1])
        right = tagged.filter(lambda t: t[0] == "R").map(lambda t: t[1])
        return left, right

    # ------------------------------------------------------------------ execution
    def execute(self, job_name: str = "flink_jpmml_amd job", restore: Optional[str] = None) -> JobExecutionResult:
        """Run the job. ``restore`` resumes from a checkpoint manifest; without one a job started by
        the restart supervisor (:mod:`flink_jpmml_amd.launch`) resumes from ``FJA_RESTORE``."""
        if restore is None:
            restore = os.environ.get("FJA_RESTORE") or None
        sinks, self._sinks = self._sinks, []
        if not sinks:
            raise RuntimeError("no sinks defined: nothing to execute")
        srv = None
        port = int(getattr(self.config, "metrics_port", 0) or 0)
        if port > 0:  # Prometheus scrape endpoint per rank for the job's lifetime
            from ..utils.metrics import METRICS

            rank = self.dist_ctx.rank if self.dist_ctx is not None else 0
            srv = METRICS.serve_prometheus(port + rank, labels={"rank": str(rank), "job": job_name})
        try:
            return Executor(self, sinks, restore).run(job_name)
        finally:
            if srv is not None:
                srv.shutdown()
                srv.server_close()


class DataStream:
    def __init__(self, env: StreamExecutionEnvironment, node: Node):
        self.env = env
        self.node = node

    def _one(self, kind: str, fn: Any, name: str, partition: str = "forward",
             parallelism: Optional[int] = None) -> "DataStream":
        p = parallelism or self.env.parallelism
        part = partition if p == self.node.parallelism else ("rebalance" if partition == "forward" else partition)
        node = Node("one", name, p, factory=fn, inputs=[(self.node, part)], uid=_uid(self.env, name), op_kind=kind)
        return DataStream(self.env, node)

    def map(self, fn: Any, name: str = "map") -> "DataStream":  # noqa: A003
        return self._one("map", fn, name)

    def filter(self, fn: Any, name: str = "filter") -> "DataStream":  # noqa: A003
        return self._one("filter", fn, name)

    def flat_map(self, fn: Any, name: str = "flat_map") -> "DataStream":
        return self._one("flat_map", fn, name)

    flatMap = flat_map  # noqa: N815

    def unbatch(self) -> "DataStream":
        """``(PredictionBatch, RecordBatch)`` elements → per-record ``(Prediction, vector)``
        (materialises Prediction objects: for sinks that need the reference's element type). A
        batch built by :meth:`to_batches` pairs each Prediction with its original event."""
        from ..api.batch import PredictionBatch

        def explode(x):
            if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], PredictionBatch):
                preds, batch = x
                rows = batch.payload if getattr(batch, "payload", None) is not None else batch
                return list(zip(preds.predictions(), rows))
            if isinstance(x, PredictionBatch):
                return x.predictions()
            return [x]

        return self._one("flat_map", explode, "unbatch")

    def to_batches(self, extract: Optional[Callable[[Any], Any]] = None, batch_rows: int = 65536,
                   model_id: Optional[Callable[[Any], str]] = None, keep_events: bool = True,
                   max_latency_ms: Optional[float] = None) -> "DataStream":
        """Per-record events → columnar :class:`~flink_jpmml_amd.api.batch.RecordBatch` elements
        (the vectorised adapter in front of the GPU path): ``extract(event)`` gives the event's
        feature row in the model's active-field order (a DenseVector, sequence or array; default:
        the event itself), ``model_id(event)`` its serving id (dynamic mode, ``BaseEvent.modelId``).
        A batch is emitted every ``batch_rows`` events, at checkpoint barriers, at end of input and
        — with ``max_latency_ms`` — when its oldest event has waited that long. The original events
        ride along as the batch ``payload`` (``unbatch()`` pairs each prediction with its event)."""
        from .operators import ToBatchesFunction

        op = ToBatchesFunction(extract, batch_rows, model_id, keep_events, max_latency_ms)
        return self._one("flat_map", op, "to_batches")

    toBatches = to_batches  # noqa: N815

    def set_parallelism(self, p: int) -> "DataStream":
        self.node.parallelism = int(p)
        return self

    def uid(self, uid: str) -> "DataStream":
        """Stable operator id (names its state in checkpoint manifests)."""
        self.node.uid = uid
        return self

    def rebalance(self) -> "DataStream":
        return _Partitioned(self, "rebalance")

    def broadcast(self) -> "DataStream":
        _mark_replicated(self.node)
        return _Partitioned(self, "broadcast")

    def connect(self, other: "DataStream") -> "ConnectedStreams":
        return ConnectedStreams(self, other)

    def add_sink(self, sink: Any) -> Node:
        if callable(sink) and not isinstance(sink, SinkFunction):
            sink = _FnSink(sink)
        node = Node("sink", "sink", 1, factory=sink, inputs=[(self.node, "rebalance" if self.node.parallelism != 1
                                                                  else "forward")], uid=_uid(self.env, "sink"),
                    op_kind="sink")
        self.env._sinks.append(node)
        return node

    addSink = add_sink  # noqa: N815

    def write_as_text(self, path: str, fmt: Optional[Callable[[Any], str]] = None) -> Node:
        """Streaming text sink (``writeAsText``): the file grows as results arrive."""
        return self.add_sink(TextSink(path, fmt))

    writeAsText = write_as_text  # noqa: N815

    def collect(self, job_name: str = "collect", restore: Optional[str] = None) -> List[Any]:
        """Attach a collecting sink, run the job, return the outputs. Under data parallelism every
        rank returns every rank's outputs, concatenated in rank order (all-gather, F5)."""
        sink = CollectSink()
        self.add_sink(sink)
        self.env.execute(job_name, restore=restore)
        if self.env.is_distributed:
            from ..parallel.dist import all_gather_object

            ctx = self.env.dist_ctx
            parts = all_gather_object(sink.values, ctx, group=ctx.group("ctrl"))
            return [x for part in parts for x in part]
        return sink.values

    executeAndCollect = collect  # noqa: N815

    # ------------------------------------------------------------------ scoring DSL (C1)
    def with_support_stream(self, support: "DataStream") -> "ConnectedStreams":
        """``stream.connect(supportStream.broadcast)`` (`S/package.scala:63-65`)."""
        return ConnectedStreams(self, support.broadcast())

    withSupportStream = with_support_stream  # noqa: N815

    def evaluate(self, model_reader: ModelReader, f: Callable[[Any, Any], Any], batch_size: Optional[int] = None,
                 device: Any = None, plan_opts: Optional[dict] = None,
                 config: Optional[ScoringConfig] = None) -> "DataStream":
        """``stream.flatMap(EvaluationFunction(reader){ out.collect(f(value, evaluator)) })``
        (`S/package.scala:76-82`)."""
        op = EvaluationFunction(model_reader, f, batch_size, device, plan_opts, config)
        return self._one("flat_map", op, "evaluate")

    def quick_evaluate(self, model_reader: ModelReader, batch_size: Optional[int] = None, device: Any = None,
                       plan_opts: Optional[dict] = None, config: Optional[ScoringConfig] = None) -> "DataStream":
        """Vector stream → ``(Prediction, vector)`` (`S/package.scala:138-142`); RecordBatch stream
        → ``(PredictionBatch, RecordBatch)``."""
        op = QuickEvaluationFunction(model_reader, batch_size, device, plan_opts, config)
        return self._one("flat_map", op, "quick_evaluate")

    quickEvaluate = quick_evaluate  # noqa: N815


def _mark_replicated(node: Node) -> None:
    """A broadcast edge: the source feeding it is read by every rank (control streams)."""
    seen = set()
    stack = [node]
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if n.kind == "source":
            if n.dist_mode == "shard":
                n.dist_mode = "replicate"
            continue
        stack.extend(up for up, _ in n.inputs)


class _Partitioned(DataStream):
    def __init__(self, stream: DataStream, partition: str):
        super().__init__(stream.env, stream.node)
        self.partition = partition


class ConnectedStreams:
    def __init__(self, first: DataStream, second: DataStream):
        self.first = first
        self.second = second
        self.env = first.env

    def process(self, fn: CoProcessFunction, name: str = "co_process") -> DataStream:
        p = self.env.parallelism
        p1 = getattr(self.first, "partition", "forward" if self.first.node.parallelism == p else "rebalance")
        p2 = getattr(self.second, "partition", "forward" if self.second.node.parallelism == p else "rebalance")
        node = Node("two", name, p, factory=fn, inputs=[(self.first.node, p1), (self.second.node, p2)],
                    uid=_uid(self.env, name), op_kind="co_process")
        return DataStream(self.env, node)

    def evaluate(self, f: Callable[[Any, Any], Any], batch_size: Optional[int] = None, device: Any = None,
                 cache_capacity: Optional[int] = None, plan_opts: Optional[dict] = None, uid: Optional[str] = None,
                 config: Optional[ScoringConfig] = None) -> DataStream:
        """Dynamic multi-model serving (`S/package.scala:107-119`). ``uid`` names the operator's
        state in checkpoints (stable across restarts)."""
        op = EvaluationCoFunction(f, batch_size, device, cache_capacity, plan_opts, config)
        out = self.process(op, "evaluate_co")
        if uid:
            out.node.uid = uid
        return out

    def quick_evaluate(self, device: Any = None, cache_capacity: Optional[int] = None,
                       plan_opts: Optional[dict] = None, uid: Optional[str] = None,
                       config: Optional[ScoringConfig] = None) -> DataStream:
        """Dynamic serving without a UDF — the multi-model counterpart of ``quickEvaluate``
        (`S/package.scala:107-119,138-142`). Columnar events (RecordBatch with ``model_id`` or
        per-row ``model_ids``) → ``(PredictionBatch, RecordBatch)`` with one prediction per row in
        row order, however many models the batch mixes (grouped device pass,
        :mod:`flink_jpmml_amd.runtime.grouped`); per-record events exposing ``to_vector()`` →
        ``(Prediction, event)``."""
        op = EvaluationCoFunction(_quick_event_udf, None, device, cache_capacity, plan_opts, config)
        op.grouped = True
        out = self.process(op, "quick_evaluate_co")
        if uid:
            out.node.uid = uid
        return out

    quickEvaluate = quick_evaluate  # noqa: N815


def _quick_event_udf(event: Any, model: Any) -> Tuple[Any, Any]:
    to_vector = getattr(event, "to_vector", None) or getattr(event, "toVector", None)
    if to_vector is None:
        raise TypeError(f"quick_evaluate on connected streams needs RecordBatch events or events with "
                        f"to_vector(), got {type(event).__name__}")
    return model.predict(to_vector()), event


__all__ = ["CollectSink", "ConnectedStreams", "DataStream", "FileSink", "SimulatedFailure",
           "StreamExecutionEnvironment", "TextSink"]
