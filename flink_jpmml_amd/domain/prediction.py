"""Prediction result ADT: ``Prediction(Score(d) | EmptyScore)``.

Reference: `S/models/prediction/Prediction.scala:30-72` and `S/models/prediction/Target.scala:25-84`.
Per-record failures are mapped to a *shared* ``Prediction(EmptyScore)`` and logged by cause; the
job never fails because of one bad record.
"""

from __future__ import annotations

import logging
import math
from typing import Callable, Union

from ..api.exceptions import (
    EvaluationException,
    InputPreparationException,
    InputValidationException,
    JPMMLExtractionException,
    NoSuchElementException,
)

logger = logging.getLogger(__name__)


class Target:
    """Sealed base of ``Score`` / ``EmptyScore`` (`S/models/prediction/Target.scala:44-58`)."""

    __slots__ = ()

    @staticmethod
    def apply(value: float) -> "Score":
        return Score(float(value))

    @staticmethod
    def empty() -> "_EmptyScore":
        return EmptyScore

    def get(self) -> float:  # pragma: no cover - overridden
        raise NotImplementedError

    def get_or_else(self, default: float) -> float:
        raise NotImplementedError

    # camelCase aliases for users switching from the Scala API
    def getOrElse(self, default: float) -> float:  # noqa: N802
        return self.get_or_else(default)

    @property
    def is_empty(self) -> bool:
        return self is EmptyScore


class Score(Target):
    """A defined score (`S/models/prediction/Target.scala:64-71`)."""

    __slots__ = ("value",)

    def __init__(self, value: float):
        self.value = float(value)

    def get(self) -> float:
        return self.value

    def get_or_else(self, default: float) -> float:
        return self.value

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, Score):
            return NotImplemented
        return self.value == other.value or (math.isnan(self.value) and math.isnan(other.value))

    def __hash__(self) -> int:
        return hash(("Score", self.value))

    def __repr__(self) -> str:
        return f"Score({self.value!r})"


class _EmptyScore(Target):
    """No score could be produced (`S/models/prediction/Target.scala:76-84`)."""

    __slots__ = ()
    _instance: "_EmptyScore | None" = None

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def get(self) -> float:
        raise NoSuchElementException("EmptyScore.nan")

    def get_or_else(self, default: float) -> float:
        return default

    def __repr__(self) -> str:
        return "EmptyScore"

    def __reduce__(self):
        return (_EmptyScore, ())


EmptyScore = _EmptyScore()


class Prediction:
    """``case class Prediction(value: Target)`` (`S/models/prediction/Prediction.scala:72`).

    ``outputs`` optionally carries the model's PMML ``<Output>`` fields; the reference extracts
    them but drops them (`S/api/pipeline/Pipeline.scala:69-70`), we expose them. They do not take
    part in equality so that goldens written against the reference compare equal."""

    __slots__ = ("value", "outputs")

    def __init__(self, value: Target, outputs: dict | None = None):
        self.value = value
        self.outputs = outputs

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, Prediction):
            return NotImplemented
        return self.value == other.value

    def __hash__(self) -> int:
        return hash(("Prediction", self.value))

    def __repr__(self) -> str:
        return f"Prediction({self.value!r})"

    # ------------------------------------------------------------------ factory
    @staticmethod
    def extract_prediction(out: Union[float, BaseException, Callable[[], float]]) -> "Prediction":
        """``Try[Double] => Prediction`` (`S/models/prediction/Prediction.scala:37-40`).

        Accepts a value (Success), an exception instance (Failure) or a thunk evaluated under
        a Try."""
        if callable(out):
            try:
                out = out()
            except Exception as e:  # NonFatal
                return Prediction.on_failed_prediction(e)
        if isinstance(out, BaseException):
            return Prediction.on_failed_prediction(out)
        return Prediction(Score(out))

    @staticmethod
    def on_failed_prediction(err: BaseException) -> "Prediction":
        """Log by failure class and return the shared empty prediction
        (`S/models/prediction/Prediction.scala:47-62`)."""
        from ..utils.metrics import METRICS

        if isinstance(err, JPMMLExtractionException):
            cause = "extraction"
            logger.warning("Error while extracting results: %s", err)
        elif isinstance(err, InputPreparationException):
            cause = "preparation"
            logger.warning("Error while preparing input: %s", err)
        elif isinstance(err, InputValidationException):
            cause = "validation"
            logger.warning("Error while validate input: %s", err)
        elif isinstance(err, EvaluationException):
            cause = "evaluation"
            logger.warning("Error while evaluate model: %s", err)
        elif isinstance(err, (TypeError, ValueError)):  # ClassCastException analogue
            cause = "target_cast"
            logger.error("Error while extract target: %s", err)
        else:
            cause = "other"
            logger.error("Error: %r", err)
        METRICS.inc(f"scoring.empty_score.{cause}")  # EmptyScore counts by failure cause
        return EMPTY_PREDICTION

    extractPrediction = extract_prediction  # noqa: N815 - Scala-style alias


EMPTY_PREDICTION = Prediction(EmptyScore)
