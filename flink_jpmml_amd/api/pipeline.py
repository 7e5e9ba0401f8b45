"""Pipeline helper steps mixed into :class:`PmmlModel` (`S/api/pipeline/Pipeline.scala:37-98`)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Optional, Tuple, Union

from .exceptions import InputPreparationException


@dataclass(frozen=True)
class FieldValue:
    """A prepared input value (JPMML ``FieldValue`` analogue): the decoded value and its numeric
    device encoding (string categories → vocabulary code, missing → NaN)."""

    value: Any
    encoded: float
    data_type: Optional[str] = None
    optype: Optional[str] = None

    @property
    def is_missing(self) -> bool:
        return self.value is None


class Pipeline:
    """Self-type mixin: relies on ``self.evaluator`` (an ``Evaluator``)."""

    def prepare_and_emit(self, outcome: Union[FieldValue, BaseException], field: str) -> Tuple[str, FieldValue]:
        """Emit the prepared value or raise :class:`InputPreparationException`
        (`S/api/pipeline/Pipeline.scala:49-54`)."""
        if isinstance(outcome, BaseException):
            raise InputPreparationException(f"The {field} field preparation failed.") from outcome
        return field, outcome

    def extract_target_fields(self, evaluation_result: Dict[str, Any]) -> List[Tuple[str, Any]]:
        return self.extract_fields(self.evaluator.model.target_fields, evaluation_result)

    def extract_output_fields(self, evaluation_result: Dict[str, Any]) -> List[Tuple[str, Any]]:
        return self.extract_fields(self.evaluator.model.output_fields, evaluation_result)

    def extract_fields(self, fields: Iterable[Optional[str]], evaluation_result: Dict[str, Any]) -> List[Tuple[str, Any]]:
        """``name -> decoded value`` for every named field (null names dropped,
        `S/api/pipeline/Pipeline.scala:79-85`)."""
        return [(f, evaluation_result.get(f)) for f in fields if f is not None]

    @staticmethod
    def extract_target_value(target: Any) -> Optional[float]:
        """String → ``float(s)`` (ValueError is the NumberFormatException analogue), numbers as-is,
        anything else → None (`S/api/pipeline/Pipeline.scala:93-98`)."""
        if isinstance(target, str):
            return float(target)
        if isinstance(target, bool):
            return None
        if isinstance(target, (int, float)):
            return float(target)
        return None

    # Scala-style aliases
    prepareAndEmit = prepare_and_emit  # noqa: N815
    extractTargetFields = extract_target_fields  # noqa: N815
    extractOutputFields = extract_output_fields  # noqa: N815
