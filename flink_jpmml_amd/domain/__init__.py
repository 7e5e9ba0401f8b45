"""L1 domain/protocol types (mirror of the reference's `S/models/` package)."""

from .checkpoint import MetadataCheckpoint, STATE_NAME
from .control import AddMessage, DelMessage, ServingMessage
from .events import BaseEvent, event_model_id
from .model_id import ModelId, ModelInfo, java_string_hash
from .prediction import EMPTY_PREDICTION, EmptyScore, Prediction, Score, Target

__all__ = [
    "AddMessage",
    "BaseEvent",
    "DelMessage",
    "EMPTY_PREDICTION",
    "EmptyScore",
    "MetadataCheckpoint",
    "ModelId",
    "ModelInfo",
    "Prediction",
    "STATE_NAME",
    "Score",
    "ServingMessage",
    "Target",
    "event_model_id",
    "java_string_hash",
]
