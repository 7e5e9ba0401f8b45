"""Flink-shaped streaming runtime + the scoring DSL (reference layers L5/L6: `S/package.scala`,
`S/api/functions/`)."""

from .clock import ManualClock, SystemClock
from .datastream import CollectSink, ConnectedStreams, DataStream, FileSink, StreamExecutionEnvironment
from .functions import (
    CheckpointedFunction,
    CoProcessFunction,
    Collector,
    FlatMapFunction,
    RichFlatMapFunction,
    SinkFunction,
    SourceContext,
    SourceFunction,
)
from .operators import EvaluationCoFunction, EvaluationFunction, ModelCache, QuickEvaluationFunction
from .runtime import JobExecutionException, JobExecutionResult, SimulatedFailure, ensure_serializable
from .sources import BatchSource, CollectionSource, GeneratorSource, ReplicatedSource, TextBatchSource, ThreadedSource

__all__ = [
    "BatchSource", "CollectionSource", "FileSink", "GeneratorSource", "ManualClock", "ReplicatedSource",
    "SystemClock", "TextBatchSource", "ThreadedSource",
    "CheckpointedFunction", "CoProcessFunction", "CollectSink", "Collector", "ConnectedStreams", "DataStream",
    "EvaluationCoFunction", "EvaluationFunction", "FlatMapFunction", "JobExecutionException", "JobExecutionResult",
    "ModelCache", "QuickEvaluationFunction", "RichFlatMapFunction", "SimulatedFailure", "SinkFunction",
    "SourceContext", "SourceFunction", "StreamExecutionEnvironment", "ensure_serializable",
]
