"""Operator state + checkpoint storage.

The reference keeps its serving metadata in a Flink *union* ``ListState`` named
``"metadata-snapshot"`` (`S/api/functions/EvaluationCoFunction.scala:84-88`): on restore every
subtask receives the union of all subtasks' entries. :class:`OperatorStateStore` reproduces that,
and :class:`CheckpointStorage` persists completed checkpoints as JSON manifests (PMML stays the
model format — a checkpoint only points at model paths).
"""

from __future__ import annotations

import json
import os
import tempfile
import time
from typing import Any, Callable, Dict, Iterable, List, Optional


class ListState:
    def __init__(self, name: str, initial: Optional[List[Any]] = None):
        self.name = name
        self._items: List[Any] = list(initial or [])

    def get(self) -> List[Any]:
        return list(self._items)

    def add(self, item: Any) -> None:
        self._items.append(item)

    def add_all(self, items: Iterable[Any]) -> None:
        self._items.extend(items)

    def update(self, items: Iterable[Any]) -> None:
        self._items = list(items)

    def clear(self) -> None:
        self._items = []


class OperatorStateStore:
    """Per-subtask store; ``restored`` holds ``name -> [items of every subtask]`` (union mode) or
    this subtask's own items (split mode)."""

    def __init__(self, restored: Optional[Dict[str, List[Any]]] = None):
        self._restored = restored or {}
        self.states: Dict[str, ListState] = {}
        self.modes: Dict[str, str] = {}

    def get_union_list_state(self, name: str) -> ListState:
        st = self.states.get(name)
        if st is None:
            st = ListState(name, self._restored.get(name, []))
            self.states[name] = st
            self.modes[name] = "union"
        return st

    def get_list_state(self, name: str) -> ListState:
        st = self.states.get(name)
        if st is None:
            st = ListState(name, self._restored.get(name, []))
            self.states[name] = st
            self.modes[name] = "split"
        return st

    getUnionListState = get_union_list_state  # noqa: N815
    getListState = get_list_state  # noqa: N815

    def snapshot(self, encode: Callable[[Any], Any]) -> Dict[str, dict]:
        return {n: {"mode": self.modes[n], "items": [encode(x) for x in st.get()]} for n, st in self.states.items()}


class CheckpointStorage:
    """Directory of ``chk-<id>.json`` manifests written atomically (tmp + rename)."""

    def __init__(self, directory: Optional[str] = None):
        self.directory = directory or tempfile.mkdtemp(prefix="fja-ckpt-")
        os.makedirs(self.directory, exist_ok=True)

    def write(self, checkpoint_id: int, payload: dict) -> str:
        payload = dict(payload, checkpoint_id=checkpoint_id, timestamp=int(time.time() * 1000))
        path = os.path.join(self.directory, f"chk-{checkpoint_id:06d}.json")
        tmp = path + ".tmp"
        with open(tmp, "w") as fh:
            json.dump(payload, fh, indent=1, sort_keys=True)
        os.replace(tmp, path)
        return path

    def latest(self) -> Optional[str]:
        files = sorted(f for f in os.listdir(self.directory) if f.startswith("chk-") and f.endswith(".json"))
        return os.path.join(self.directory, files[-1]) if files else None

    @staticmethod
    def read(path: str) -> dict:
        with open(path) as fh:
            return json.load(fh)
