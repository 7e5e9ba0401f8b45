"""Serialized operator state of dynamic serving: the *metadata* table only.

Reference: `S/models/state/CheckpointType.scala:29-32` (``java.util.HashMap[ModelId, ModelInfo]``
held in a union ``ListState`` named ``"metadata-snapshot"``). Models themselves are never
checkpointed; they are re-read lazily by path after restore (`README.md:89-92`).

Our on-disk form is JSON: ``{"name": "metadata-snapshot", "entries": [{"name", "version",
"path", "sha256"?}]}``. PMML stays the model format, this file only points at it.
"""

from __future__ import annotations

import json
from typing import Dict, Iterable, List, Mapping

from .model_id import ModelId, ModelInfo

STATE_NAME = "metadata-snapshot"

MetadataCheckpoint = Dict[ModelId, ModelInfo]
MetadataCheckpointedList = List[MetadataCheckpoint]


def metadata_to_json(meta: Mapping[ModelId, ModelInfo]) -> list:
    return [
        {"name": k.name, "version": k.version, "path": v.path}
        for k, v in sorted(meta.items(), key=lambda kv: (kv[0].name, kv[0].version))
    ]


def metadata_from_json(entries: Iterable[dict]) -> MetadataCheckpoint:
    return {ModelId(e["name"], int(e["version"])): ModelInfo(e["path"]) for e in entries}


def union_restore(snapshots: Iterable[Mapping[ModelId, ModelInfo]]) -> MetadataCheckpoint:
    """Union of every subtask's snapshot (`S/api/functions/EvaluationCoFunction.scala:90-95`)."""
    out: MetadataCheckpoint = {}
    for snap in snapshots:
        out.update(snap)
    return out


def dumps(meta: Mapping[ModelId, ModelInfo]) -> str:
    return json.dumps({"name": STATE_NAME, "entries": metadata_to_json(meta)}, indent=1)


def loads(text: str) -> MetadataCheckpoint:
    doc = json.loads(text)
    return metadata_from_json(doc.get("entries", []))
