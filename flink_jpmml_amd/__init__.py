"""flink_jpmml_amd — an MI355X-native streaming PMML scoring engine.

Same capabilities as flink-jpmml (Flink-shaped operator DSL over PMML models, dynamic
multi-model serving driven by Add/Del control messages, metadata checkpoints), re-designed for
AMD Instinct MI355X: models are parsed once, compiled into device tensors and scored in
micro-batches by hand-written CDNA4 HIP kernels; the stream is sharded data-parallel across the
GPUs of a node with RCCL over xGMI.
"""

__version__ = "0.1.0"

from .api import (  # noqa: E402
    DenseVector,
    ModelReader,
    PmmlModel,
    SparseVector,
)
from .domain import (  # noqa: E402
    AddMessage,
    DelMessage,
    EmptyScore,
    ModelId,
    ModelInfo,
    Prediction,
    Score,
    ServingMessage,
    Target,
)

__all__ = [
    "AddMessage", "DelMessage", "DenseVector", "EmptyScore", "ModelId", "ModelInfo", "ModelReader",
    "PmmlModel", "Prediction", "Score", "ServingMessage", "SparseVector", "Target", "__version__",
]
