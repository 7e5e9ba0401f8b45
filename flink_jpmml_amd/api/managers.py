"""Serving-state managers driven by control messages.

* :func:`metadata_manager` (`S/api/managers/MetadataManager.scala:41-86`): ``Add`` inserts
  ``ModelId → ModelInfo`` unless the id already exists (WARN + unchanged: an update needs a new
  version); ``Del`` removes the id. Returns a new mapping (the input is not mutated).
* :func:`models_manager` (`S/api/managers/ModelsManager.scala:41-57`): on ``Del`` returns the cache
  keys to evict. The reference keys its cache by ``"name_version".hashCode``; our cache keys by the
  exact :class:`ModelId` (no hash collisions), and this function accepts
  both key kinds.
"""

from __future__ import annotations

import logging
from typing import Any, Iterable, Mapping, Set

from ..domain.control import AddMessage, DelMessage, ServingMessage
from ..domain.model_id import ModelId, ModelInfo

logger = logging.getLogger(__name__)


def metadata_manager(command: ServingMessage, metadata: Mapping[ModelId, ModelInfo]) -> dict:
    meta = dict(metadata)
    if isinstance(command, AddMessage):
        mid = command.model_id
        if mid in meta:
            logger.warning("ADD action on existing models is not possible (newer version needed). %s given.", command)
            return meta
        meta[mid] = command.model_info
        return meta
    if isinstance(command, DelMessage):
        meta.pop(command.model_id, None)
        return meta
    raise TypeError(f"unknown control message {command!r}")


def models_manager(command: ServingMessage, cache_keys: Iterable[Any]) -> Set[Any]:
    if not isinstance(command, DelMessage):
        return set()
    mid = command.model_id
    wanted = {mid, mid.java_hash_code, mid.identifier}
    return {k for k in cache_keys if k in wanted}


class MetadataManager:
    """Type-class style entry point: ``MetadataManager(cmd, metadata)``."""

    def __new__(cls, command: ServingMessage, metadata: Mapping[ModelId, ModelInfo]):  # type: ignore[misc]
        return metadata_manager(command, metadata)


class ModelsManager:
    def __new__(cls, command: ServingMessage, cache_keys: Iterable[Any]):  # type: ignore[misc]
        return models_manager(command, cache_keys)
