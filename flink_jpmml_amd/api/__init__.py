"""L2/L3 public API: model handle, reader, vectors, managers, exceptions
(mirror of the reference's `S/api/` package)."""

from .converter import PmmlInput, vector_conversion
from .evaluator import EMPTY_EVALUATOR, EmptyEvaluator, Evaluator, PmmlEvaluator
from .exceptions import (
    EmptyEvaluatorException,
    EvaluationException,
    InputPreparationException,
    InputValidationException,
    JPMMLExtractionException,
    ModelLoadingException,
    NoSuchElementException,
    PmmlParseError,
    UnsupportedFeatureException,
    WrongModelIdFormat,
)
from .managers import MetadataManager, ModelsManager, metadata_manager, models_manager
from .pipeline import FieldValue
from .pmml_model import PmmlModel
from .reader import FsReader, ModelReader
from .vectors import DenseVector, SparseVector, Vector, pack_vectors

__all__ = [
    "DenseVector", "EMPTY_EVALUATOR", "EmptyEvaluator", "EmptyEvaluatorException", "EvaluationException",
    "Evaluator", "FieldValue", "FsReader", "InputPreparationException", "InputValidationException",
    "JPMMLExtractionException", "MetadataManager", "ModelLoadingException", "ModelReader", "ModelsManager",
    "NoSuchElementException", "PmmlEvaluator", "PmmlInput", "PmmlModel", "PmmlParseError", "SparseVector",
    "UnsupportedFeatureException", "Vector", "WrongModelIdFormat", "metadata_manager", "models_manager",
    "pack_vectors", "vector_conversion",
]
