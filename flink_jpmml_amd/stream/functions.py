"""Flink-shaped user-function interfaces of the mini stream runtime.

Mirrors the Flink contracts the reference builds on (``RichFlatMapFunction``,
``CoProcessFunction``, ``CheckpointedFunction``, ``SourceFunction``, ``SinkFunction``) with
Python naming; camelCase aliases keep Scala-style code recognisable.
"""

from __future__ import annotations

from typing import Any, Callable, Iterable, List, Optional


class Collector:
    """Output collector handed to ``flat_map`` / ``process_element*``. ``collect_many`` hands a
    whole chunk of outputs downstream in one call (the runtime's chunked path: operators that
    implement ``flat_map_many`` / ``process_elements1`` / ``invoke_many`` receive chunks)."""

    __slots__ = ("_emit", "_emit_many")

    def __init__(self, emit: Callable[[Any], None], emit_many: Optional[Callable[[list], None]] = None):
        self._emit = emit
        self._emit_many = emit_many

    def collect(self, value: Any) -> None:
        self._emit(value)

    def collect_many(self, values: list) -> None:
        if self._emit_many is not None:
            self._emit_many(values)
        else:
            for v in values:
                self._emit(v)


class ListCollector(Collector):
    def __init__(self):
        self.items: List[Any] = []
        super().__init__(self.items.append, self.items.extend)


class RuntimeContext:
    """What an operator instance knows about where it runs: its subtask index / parallelism, the
    job's processing-time clock and timer service, the job-level scoring config and — under data
    parallelism across GPUs — the distributed context (``dist``, one subtask per rank)."""

    def __init__(self, task_name: str, subtask_index: int, parallelism: int, clock=None, dist=None,
                 config=None):
        self.task_name = task_name
        self.index_of_this_subtask = subtask_index
        self.number_of_parallel_subtasks = parallelism
        self.clock = clock
        self.dist = dist
        self.config = config

    getIndexOfThisSubtask = property(lambda self: self.index_of_this_subtask)  # noqa: N815

    def now(self) -> float:
        return self.clock.now() if self.clock is not None else __import__("time").monotonic()

    def register_timer(self, deadline: float, callback) -> None:
        """Processing-time timer: ``callback(now)`` runs on the job thread at/after ``deadline``."""
        if self.clock is not None:
            self.clock.timers.register(deadline, callback)


class RichFunction:
    runtime_context: Optional[RuntimeContext] = None

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        pass

    def close(self) -> None:
        pass

    def set_runtime_context(self, ctx: RuntimeContext) -> None:
        self.runtime_context = ctx

    def get_runtime_context(self) -> Optional[RuntimeContext]:
        return self.runtime_context


class MapFunction(RichFunction):
    def map(self, value: Any) -> Any:  # noqa: A003
        raise NotImplementedError


class FilterFunction(RichFunction):
    def filter(self, value: Any) -> bool:  # noqa: A003
        raise NotImplementedError


class FlatMapFunction(RichFunction):
    def flat_map(self, value: Any, out: Collector) -> None:
        raise NotImplementedError

    def end_of_input(self, out: Collector) -> None:
        """Called once when the input is exhausted (flush hook for micro-batching operators)."""

    def on_barrier(self, out: Collector) -> None:
        """Called before a checkpoint barrier passes the operator (flush hook)."""


RichFlatMapFunction = FlatMapFunction


class ProcessContext:
    def __init__(self, timestamp: Optional[int] = None):
        self.timestamp = timestamp


class CoProcessFunction(RichFunction):
    """Two-input operator: ``process_element1`` for events, ``process_element2`` for control."""

    def process_element1(self, value: Any, ctx: ProcessContext, out: Collector) -> None:
        raise NotImplementedError

    def process_element2(self, value: Any, ctx: ProcessContext, out: Collector) -> None:
        raise NotImplementedError

    def end_of_input(self, out: Collector) -> None:
        pass

    def on_barrier(self, out: Collector) -> None:
        pass

    # Scala-style aliases
    def processElement1(self, value, ctx, out):  # noqa: N802
        return self.process_element1(value, ctx, out)

    def processElement2(self, value, ctx, out):  # noqa: N802
        return self.process_element2(value, ctx, out)


class CheckpointedFunction:
    """Operator with managed state (`S/api/functions/EvaluationCoFunction.scala:76-96`)."""

    def snapshot_state(self, context: "FunctionSnapshotContext") -> None:
        raise NotImplementedError

    def initialize_state(self, context: "FunctionInitializationContext") -> None:
        raise NotImplementedError


class FunctionSnapshotContext:
    def __init__(self, checkpoint_id: int, timestamp: int):
        self.checkpoint_id = checkpoint_id
        self.checkpoint_timestamp = timestamp


class FunctionInitializationContext:
    def __init__(self, operator_state_store, restored: bool):
        self.operator_state_store = operator_state_store
        self._restored = restored

    def is_restored(self) -> bool:
        return self._restored

    isRestored = is_restored  # noqa: N815

    def get_operator_state_store(self):
        return self.operator_state_store


class SourceContext:
    """Handed to ``SourceFunction.run``; ``collect`` pushes one element downstream."""

    def __init__(self, emit: Callable[[Any], None], lock=None):
        self._emit = emit
        self._lock = lock

    def collect(self, value: Any) -> None:
        self._emit(value)

    def get_checkpoint_lock(self):
        return self._lock


class SourceFunction:
    """A (possibly unbounded) source. ``run`` must return when the source is exhausted or
    ``cancel`` was called. Sources that can be split across parallel subtasks implement
    :meth:`split`."""

    def run(self, ctx: SourceContext) -> None:
        raise NotImplementedError

    def cancel(self) -> None:
        pass

    def iterate(self) -> Iterable[Any]:
        """Pull-style iteration. Sources that only implement ``run(ctx)`` are run on a thread of
        their own by the runtime (:class:`flink_jpmml_amd.stream.sources.ThreadedSource`); this
        default exists for direct callers and drains a finite ``run``."""
        buf: List[Any] = []
        self.run(SourceContext(buf.append))
        return iter(buf)


class SinkFunction:
    """Sink contract. Transactional sinks (exactly-once across restarts) also implement
    ``pre_commit(checkpoint_id)`` — make everything received so far durable but invisible —
    ``commit(checkpoint_id)`` — publish it once the checkpoint manifest is written — and
    ``recover()`` — drop what a crashed run pre-committed but never committed."""

    def invoke(self, value: Any) -> None:
        raise NotImplementedError

    def open(self, context: Optional[RuntimeContext] = None) -> None:  # noqa: A003
        pass

    def close(self) -> None:
        pass
