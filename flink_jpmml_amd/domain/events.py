"""Event contract for dynamic (multi-model) serving.

Reference: `S/models/input/BaseEvent.scala:25-31` — every event routed through
``with_support_stream(...).evaluate(...)`` carries the ``model_id`` string of the model that must
score it and an ``occurred_on`` timestamp.
"""

from __future__ import annotations

from typing import Protocol, runtime_checkable


@runtime_checkable
class BaseEvent(Protocol):
    @property
    def model_id(self) -> str: ...

    @property
    def occurred_on(self) -> int: ...


def event_model_id(event) -> str:
    """Read the model id of an event; accepts ``model_id`` or Scala-style ``modelId``."""
    mid = getattr(event, "model_id", None)
    if mid is None:
        mid = getattr(event, "modelId", None)
    if mid is None:
        raise AttributeError(f"{type(event).__name__} does not carry a model_id (see BaseEvent)")
    return mid
