"""``Evaluator`` ADT: ``PmmlEvaluator(compiled)`` | ``EmptyEvaluator``.

Reference: `S/api/Evaluator.scala:29-91`. ``EmptyEvaluator.model`` raises
:class:`EmptyEvaluatorException`; it backs the placeholder model handed to UDFs for events whose
model id is unknown (`S/api/functions/EvaluationCoFunction.scala:106-110`).
"""

from __future__ import annotations

from typing import Any

from .exceptions import EmptyEvaluatorException


class Evaluator:
    @staticmethod
    def apply(model: Any) -> "PmmlEvaluator":
        return PmmlEvaluator(model)

    @staticmethod
    def empty() -> "EmptyEvaluator":
        return EMPTY_EVALUATOR

    @property
    def model(self):  # pragma: no cover - overridden
        raise NotImplementedError

    def get_or_else(self, default: Any) -> Any:
        raise NotImplementedError

    getOrElse = get_or_else  # noqa: N815


class PmmlEvaluator(Evaluator):
    __slots__ = ("_model",)

    def __init__(self, model: Any):
        self._model = model

    @property
    def model(self):
        return self._model

    def get_or_else(self, default: Any) -> Any:
        return self._model

    def __eq__(self, other: object) -> bool:
        return isinstance(other, PmmlEvaluator) and other._model is self._model

    def __hash__(self) -> int:
        return id(self._model)

    def __repr__(self) -> str:
        return f"PmmlEvaluator({getattr(self._model, 'model_name', '?')!r})"


class EmptyEvaluator(Evaluator):
    @property
    def model(self):
        raise EmptyEvaluatorException("EmptyEvaluator has no model")

    def get_or_else(self, default: Any) -> Any:
        return default

    def __repr__(self) -> str:
        return "EmptyEvaluator"


EMPTY_EVALUATOR = EmptyEvaluator()
