"""Model identity: ``ModelId(name, version)`` and ``ModelInfo(path)``.

Reference: `S/models/core/ModelId.scala:32-64`, `S/models/core/ModelInfo.scala:26`.
An identifier is ``"<lowercase-uuid>_<digits>"``; a malformed identifier raises
:class:`WrongModelIdFormat` (fatal in the dynamic operator, as in the reference).
"""

from __future__ import annotations

import re
from dataclasses import dataclass

from ..api.exceptions import WrongModelIdFormat

SEPARATOR = "_"
_NAME_RE = r"[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}"
_ID_RE = re.compile(r"\s*(" + _NAME_RE + r")\s*" + SEPARATOR + r"(\d+)")


def java_string_hash(s: str) -> int:
    """``java.lang.String.hashCode`` (signed 32-bit), used for cache-key parity with
    `S/models/core/ModelId.scala:62`."""
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        cp = ord(ch)
        if cp > 0xFFFF:  # surrogate pair, as Java stores it
            cp -= 0x10000
            for unit in (0xD800 + (cp >> 10), 0xDC00 + (cp & 0x3FF)):
                h = (31 * h + unit) & 0xFFFFFFFF
        else:
            h = (31 * h + cp) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


@dataclass(frozen=True)
class ModelId:
    name: str
    version: int

    @staticmethod
    def from_identifier(identifier: str) -> "ModelId":
        """Parse ``"<uuid>_<version>"`` (`S/models/core/ModelId.scala:47-51`)."""
        if not isinstance(identifier, str):
            raise WrongModelIdFormat(f"model id must be a string, got {type(identifier).__name__}")
        m = _ID_RE.fullmatch(identifier)
        if m is None:
            raise WrongModelIdFormat(f"`{identifier}` is not a valid <uuid>_<version> model id")
        return ModelId(m.group(1), int(m.group(2)))

    fromIdentifier = from_identifier  # noqa: N815

    @property
    def identifier(self) -> str:
        return f"{self.name}{SEPARATOR}{self.version}"

    @property
    def java_hash_code(self) -> int:
        """Equals ``(name + "_" + version).hashCode`` like the reference's override."""
        return java_string_hash(self.identifier)

    def __str__(self) -> str:
        return self.identifier


@dataclass(frozen=True)
class ModelInfo:
    """Metadata value: where the PMML document lives (`S/models/core/ModelInfo.scala:26`)."""

    path: str
