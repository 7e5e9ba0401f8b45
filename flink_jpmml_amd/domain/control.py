"""Control-stream protocol: ``AddMessage`` / ``DelMessage``.

Reference: `S/models/control/ServingMessage.scala:27-60`. ``occurred_on`` is carried but, as in
the reference, not used for ordering: control messages act in arrival order.

For the data-parallel runtime a message also has a fixed-size binary encoding
(:meth:`ServingMessage.pack`) so rank 0 can broadcast it to every GPU rank as one small tensor
(SURVEY §2.6 F1).
"""

from __future__ import annotations

import struct
import uuid as _uuid
from dataclasses import dataclass

from .model_id import ModelId, ModelInfo

_OP_ADD = 1
_OP_DEL = 2


@dataclass(frozen=True)
class ServingMessage:
    name: str
    version: int
    occurred_on: int

    @property
    def model_id(self) -> ModelId:
        return ModelId(self.name, int(self.version))

    # camelCase alias (Scala API parity)
    @property
    def modelId(self) -> ModelId:  # noqa: N802
        return self.model_id

    # --------------------------------------------------------------- wire format
    def pack(self) -> bytes:
        """Encode as ``[op u8][uuid 16B][version i64][occurred_on i64][path_len u32][path utf8]``."""
        op = _OP_ADD if isinstance(self, AddMessage) else _OP_DEL
        path = getattr(self, "path", "").encode("utf-8")
        try:
            name_bytes = _uuid.UUID(self.name).bytes
            raw_name = b""
        except ValueError:  # non-uuid names are carried verbatim
            name_bytes = b"\x00" * 16
            raw_name = self.name.encode("utf-8")
        return (
            struct.pack("<B16sqqII", op, name_bytes, int(self.version), int(self.occurred_on), len(path), len(raw_name))
            + path
            + raw_name
        )

    @staticmethod
    def unpack(buf: bytes) -> "ServingMessage":
        op, name_bytes, version, occurred, plen, nlen = struct.unpack_from("<B16sqqII", buf, 0)
        off = struct.calcsize("<B16sqqII")
        path = buf[off : off + plen].decode("utf-8")
        off += plen
        name = buf[off : off + nlen].decode("utf-8") if nlen else str(_uuid.UUID(bytes=name_bytes))
        if op == _OP_ADD:
            return AddMessage(name, version, path, occurred)
        if op == _OP_DEL:
            return DelMessage(name, version, occurred)
        raise ValueError(f"unknown control opcode {op}")


@dataclass(frozen=True, init=False)
class AddMessage(ServingMessage):
    path: str

    def __init__(self, name: str, version: int, path: str, occurred_on: int = 0):
        object.__setattr__(self, "name", name)
        object.__setattr__(self, "version", int(version))
        object.__setattr__(self, "path", path)
        object.__setattr__(self, "occurred_on", int(occurred_on))

    @property
    def model_info(self) -> ModelInfo:
        return ModelInfo(self.path)

    @property
    def modelInfo(self) -> ModelInfo:  # noqa: N802
        return self.model_info


@dataclass(frozen=True, init=False)
class DelMessage(ServingMessage):
    def __init__(self, name: str, version: int, occurred_on: int = 0):
        object.__setattr__(self, "name", name)
        object.__setattr__(self, "version", int(version))
        object.__setattr__(self, "occurred_on", int(occurred_on))
