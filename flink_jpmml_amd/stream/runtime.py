"""A small deterministic dataflow runtime with Flink's operator semantics.

The reference runs on Apache Flink (TaskManagers, network stack, checkpoints). This runtime keeps
exactly the semantics the reference's operators depend on, in one process:

* a job graph of sources, one-input operators (map / flat_map / filter / process), two-input
  operators (``connect`` + ``broadcast``) and sinks;
* per-operator **parallelism**: every subtask holds its own (deep-copied) operator instance —
  one model replica per subtask, like Flink (`S/api/functions/EvaluationFunction.scala:43`);
  records are routed ``forward`` / ``rebalance`` (round-robin) / ``broadcast``;
* **deterministic interleaving** of multiple sources: elements are merged by timestamp when the
  sources provide one, else by source order — the analogue of the reference's
  ``TemporizedSourceFunction`` (`T/sources/TemporizedSourceFunction.scala:35-56`) without sleeps;
* **checkpoints**: count-based barriers; ``CheckpointedFunction``s snapshot into operator state
  (union / split list state) persisted as JSON by :class:`CheckpointStorage`; ``execute(restore=…)``
  re-initialises operators from a manifest (`S/api/functions/EvaluationCoFunction.scala:76-96`);
* failures inside operators abort the job with :class:`JobExecutionException` (as Flink's
  ``JobExecutionException`` in the reference's tests, `T/RichDataStreamSpec.scala:82-89`).
"""

from __future__ import annotations

import copy
import heapq
import itertools
import logging
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple

from .functions import (
    CheckpointedFunction,
    CoProcessFunction,
    Collector,
    FunctionInitializationContext,
    FunctionSnapshotContext,
    ProcessContext,
    RichFunction,
    RuntimeContext,
    SinkFunction,
    SourceFunction,
)
from .state import CheckpointStorage, OperatorStateStore

logger = logging.getLogger(__name__)


class JobExecutionException(RuntimeError):
    """The job failed; ``__cause__`` is the operator's exception."""


class SimulatedFailure(RuntimeError):
    """Raised by the fault-injection hook (:meth:`StreamExecutionEnvironment.inject_failure`)."""


_uid = itertools.count()


@dataclass
class Node:
    kind: str  # source | one | two | sink
    name: str
    parallelism: int
    factory: Any = None  # operator prototype (deep-copied per subtask)
    inputs: List[Tuple["Node", str]] = field(default_factory=list)  # (upstream, partitioning)
    source: Any = None
    timestamp_fn: Optional[Callable[[Any], Any]] = None
    uid: str = ""
    op_kind: str = ""  # map | flat_map | filter | process | co_process | sink

    def __hash__(self) -> int:
        return id(self)


@dataclass
class JobExecutionResult:
    job_name: str
    net_runtime_ms: float
    records_in: int
    checkpoints: List[str]
    accumulators: Dict[str, Any] = field(default_factory=dict)


def _encode_state(x: Any) -> Any:
    """JSON encoding of state items: dicts keyed by ModelId become lists of entries."""
    from ..domain.model_id import ModelId, ModelInfo

    if isinstance(x, dict) and all(isinstance(k, ModelId) for k in x):
        return {"__metadata__": [{"name": k.name, "version": k.version, "path": v.path if isinstance(v, ModelInfo)
                                  else str(v)} for k, v in x.items()]}
    return x


def _decode_state(x: Any) -> Any:
    from ..domain.model_id import ModelId, ModelInfo

    if isinstance(x, dict) and "__metadata__" in x:
        return {ModelId(e["name"], int(e["version"])): ModelInfo(e["path"]) for e in x["__metadata__"]}
    return x


class _Subtask:
    def __init__(self, node: Node, index: int, op: Any):
        self.node = node
        self.index = index
        self.op = op
        self.out: Optional[Collector] = None
        self.rr = 0


class Executor:
    def __init__(self, env: "StreamExecutionEnvironment", sinks: List[Node], restore: Optional[str]):
        self.env = env
        self.sinks = sinks
        self.restore = restore
        self.nodes: List[Node] = self._topo(sinks)
        self.down: Dict[int, List[Tuple[Node, str, int]]] = {id(n): [] for n in self.nodes}
        for n in self.nodes:
            for port, (up, part) in enumerate(n.inputs):
                self.down[id(up)].append((n, part, port))
        self.subtasks: Dict[int, List[_Subtask]] = {}
        self.records_in = 0
        self.checkpoint_paths: List[str] = []

    @staticmethod
    def _topo(sinks: List[Node]) -> List[Node]:
        order: List[Node] = []
        seen = set()

        def visit(n: Node) -> None:
            if id(n) in seen:
                return
            seen.add(id(n))
            for up, _ in n.inputs:
                visit(up)
            order.append(n)

        for s in sinks:
            visit(s)
        return order

    # ------------------------------------------------------------------ setup
    def _instantiate(self) -> None:
        restored_state: Dict[str, Dict[str, list]] = {}
        if self.restore:
            doc = CheckpointStorage.read(self.restore)
            restored_state = doc.get("operators", {})
        for n in self.nodes:
            subs = []
            for i in range(n.parallelism):
                op = None
                if n.kind in ("one", "two", "sink"):
                    op = n.factory if n.parallelism == 1 and not self.env.copy_operators else _clone(n.factory)
                st = _Subtask(n, i, op)
                subs.append(st)
            self.subtasks[id(n)] = subs
            for st in subs:
                op = st.op
                if isinstance(op, RichFunction):
                    op.set_runtime_context(RuntimeContext(n.name, st.index, n.parallelism))
                if isinstance(op, CheckpointedFunction):
                    restored = None
                    snap = restored_state.get(n.uid)
                    if snap is not None:
                        restored = {}
                        for name, entries in snap.items():
                            mode = entries.get("mode", "union")
                            parts = entries.get("subtasks", [])
                            if mode == "union":
                                items = [_decode_state(x) for part in parts for x in part]
                            else:  # split: round-robin redistribution
                                flat = [_decode_state(x) for part in parts for x in part]
                                items = flat[st.index::n.parallelism]
                            restored[name] = items
                    store = OperatorStateStore(restored)
                    op._state_store = store
                    op.initialize_state(FunctionInitializationContext(store, restored is not None))
        for n in self.nodes:
            for st in self.subtasks[id(n)]:
                st.out = Collector(self._emitter(n, st))
                if isinstance(st.op, RichFunction):
                    st.op.open({})

    # ------------------------------------------------------------------ routing
    def _emitter(self, node: Node, st: _Subtask) -> Callable[[Any], None]:
        downs = self.down[id(node)]

        def emit(value: Any) -> None:
            for dn, part, port in downs:
                subs = self.subtasks[id(dn)]
                if part == "broadcast":
                    targets = subs
                elif part == "forward" and len(subs) == node.parallelism:
                    targets = [subs[st.index]]
                else:  # rebalance
                    targets = [subs[st.rr % len(subs)]]
                    st.rr += 1
                for t in targets:
                    self._deliver(dn, t, port, value)

        return emit

    def _deliver(self, node: Node, st: _Subtask, port: int, value: Any) -> None:
        op = st.op
        k = node.op_kind
        if k == "map":
            st.out.collect(op.map(value) if hasattr(op, "map") else op(value))
        elif k == "filter":
            keep = op.filter(value) if hasattr(op, "filter") else op(value)
            if keep:
                st.out.collect(value)
        elif k in ("flat_map", "process"):
            if hasattr(op, "flat_map"):
                op.flat_map(value, st.out)
            else:
                for v in op(value):
                    st.out.collect(v)
        elif k == "co_process":
            ctx = ProcessContext(None)
            if port == 0:
                op.process_element1(value, ctx, st.out)
            else:
                op.process_element2(value, ctx, st.out)
        elif k == "sink":
            op.invoke(value) if hasattr(op, "invoke") else op(value)
        else:  # pragma: no cover
            raise RuntimeError(f"unknown operator kind {k}")

    # ------------------------------------------------------------------ sources
    def _source_iter(self, n: Node) -> Iterator[Any]:
        src = n.source
        if isinstance(src, SourceFunction):
            return iter(src.iterate())
        return iter(src)

    def _merged(self) -> Iterator[Tuple[Node, Any]]:
        """Deterministic merge of every source: by timestamp when all sources define one, else
        round-robin by source (ties broken by source order)."""
        sources = [n for n in self.nodes if n.kind == "source"]
        iters = [(n, self._source_iter(n)) for n in sources]
        timed = all(n.timestamp_fn is not None for n in sources) and len(sources) > 1
        if timed:
            heap = []
            for si, (n, it) in enumerate(iters):
                for v in it:
                    heapq.heappush(heap, (n.timestamp_fn(v), si, next(_uid), n, v))
                    break
            while heap:
                _, si, _, n, v = heapq.heappop(heap)
                yield n, v
                it = iters[si][1]
                for nv in it:
                    heapq.heappush(heap, (n.timestamp_fn(nv), si, next(_uid), n, nv))
                    break
            return
        live = list(iters)
        while live:
            nxt = []
            for n, it in live:
                try:
                    v = next(it)
                except StopIteration:
                    continue
                yield n, v
                nxt.append((n, it))
            live = nxt

    # ------------------------------------------------------------------ checkpoints
    def _checkpoint(self, cid: int) -> None:
        for n in self.nodes:
            for st in self.subtasks[id(n)]:
                if hasattr(st.op, "on_barrier"):
                    st.op.on_barrier(st.out)
        operators: Dict[str, Dict[str, dict]] = {}
        for n in self.nodes:
            subs = self.subtasks[id(n)]
            if not subs or not isinstance(subs[0].op, CheckpointedFunction):
                continue
            per_state: Dict[str, dict] = {}
            for st in subs:
                st.op.snapshot_state(FunctionSnapshotContext(cid, int(time.time() * 1000)))
                snap = st.op._state_store.snapshot(_encode_state)
                for name, s in snap.items():
                    e = per_state.setdefault(name, {"mode": s["mode"], "subtasks": []})
                    e["subtasks"].append(s["items"])
            operators[n.uid] = per_state
        path = self.env.checkpoint_storage.write(cid, {"operators": operators, "records_in": self.records_in})
        self.checkpoint_paths.append(path)

    # ------------------------------------------------------------------ run
    def run(self, job_name: str) -> JobExecutionResult:
        t0 = time.perf_counter()
        try:
            self._instantiate()
            cid = 0
            every = self.env.checkpoint_every
            for n, v in self._merged():
                self.records_in += 1
                if self.env.fail_after is not None and self.records_in > self.env.fail_after:
                    raise SimulatedFailure(f"injected failure after {self.env.fail_after} records")
                for st in self.subtasks[id(n)]:
                    st.out.collect(v)
                    break  # sources have parallelism 1 in this runtime
                if every and self.records_in % every == 0:
                    cid += 1
                    self._checkpoint(cid)
            for n in self.nodes:  # end of input: flush buffered micro-batches, in topological order
                for st in self.subtasks[id(n)]:
                    if hasattr(st.op, "end_of_input"):
                        st.op.end_of_input(st.out)
        except Exception as e:  # noqa: BLE001 - any operator failure fails the job
            raise JobExecutionException(f"Job '{job_name}' failed: {type(e).__name__}: {e}") from e
        finally:
            for n in self.nodes:
                for st in self.subtasks.get(id(n), []):
                    if isinstance(st.op, (RichFunction, SinkFunction)):
                        try:
                            st.op.close()
                        except Exception:  # noqa: BLE001
                            logger.exception("close() failed")
        return JobExecutionResult(job_name, (time.perf_counter() - t0) * 1e3, self.records_in, self.checkpoint_paths)


def _clone(op: Any) -> Any:
    """Per-subtask copy of an operator; goes through cloudpickle when available so that an
    operator that could not be shipped to a remote worker fails here, like Flink's
    ``ClosureCleaner.clean(..., checkSerializable = true)``."""
    try:
        import cloudpickle

        return cloudpickle.loads(cloudpickle.dumps(op))
    except ImportError:  # pragma: no cover
        return copy.deepcopy(op)


def ensure_serializable(obj: Any) -> Any:
    import cloudpickle

    return cloudpickle.loads(cloudpickle.dumps(obj))
