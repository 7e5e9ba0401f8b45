"""Exception hierarchy of the scoring engine.

Mirrors the six reference exceptions (`S/api/exceptions/package.scala:27-53`) so that code
written against flink-jpmml keeps its error-handling structure:

* per-record failures (validation / preparation / evaluation / extraction) are caught by
  :meth:`Prediction.extract_prediction` and become ``EmptyScore`` — they never fail a job;
* :class:`ModelLoadingException` and :class:`WrongModelIdFormat` are fatal and propagate
  out of the stream operator (the job fails), exactly as in the reference
  (`S/api/functions/EvaluationFunction.scala:45-48`, `S/models/core/ModelId.scala:47-51`).
"""

from __future__ import annotations


class FlinkJpmmlError(Exception):
    """Base class of every engine-specific error."""


class InputValidationException(FlinkJpmmlError):
    """Input vector size does not match the model's active-field count
    (`S/api/PmmlModel.scala:127-134`)."""


class InputPreparationException(FlinkJpmmlError):
    """A field value could not be prepared for the model (`S/api/pipeline/Pipeline.scala:49-54`)."""


class JPMMLExtractionException(FlinkJpmmlError):
    """The evaluation produced no usable target value (`S/api/PmmlModel.scala:167-174`).

    The name is kept for API parity with the reference even though no JPMML is involved."""


# Alias with an engine-neutral name.
ExtractionException = JPMMLExtractionException


class EvaluationException(FlinkJpmmlError):
    """A model-level evaluation error (PMML semantics violated at score time); the analogue of
    JPMML's ``org.jpmml.evaluator.EvaluationException`` handled in
    `S/models/prediction/Prediction.scala:54`."""


class ModelLoadingException(FlinkJpmmlError):
    """The model could not be read / parsed / compiled. Fatal (`S/api/exceptions/package.scala:42-43`)."""

    def __init__(self, msg: str, cause: BaseException | None = None):
        super().__init__(msg)
        self.cause = cause
        if cause is not None:
            self.__cause__ = cause


class NoSuchElementException(LookupError):
    """Python analogue of ``java.util.NoSuchElementException``."""


class EmptyEvaluatorException(NoSuchElementException):
    """Raised by every operation on an empty evaluator (`S/api/exceptions/package.scala:48`)."""


class WrongModelIdFormat(IndexError):
    """A model identifier is not ``<uuid>_<version>`` (`S/api/exceptions/package.scala:53`;
    the reference extends ``ArrayIndexOutOfBoundsException``, hence ``IndexError``)."""


class PmmlParseError(FlinkJpmmlError):
    """The PMML document is malformed or uses an element this engine does not support."""


class UnsupportedFeatureException(PmmlParseError):
    """The PMML document is valid but uses a feature not implemented by this engine."""
