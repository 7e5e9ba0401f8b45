"""Model I/O: ``ModelReader(source_path)`` + file-system resolution.

Reference: `S/api/reader/ModelReader.scala:27` and `S/api/reader/FsReader.scala:32-49` —
``buildDistributedPath`` opens the path through Flink's FileSystem abstraction (local, HDFS, S3,
Alluxio) and returns the **whole document as a string**.

Here:

* plain paths and ``file://`` URLs are read directly;
* any other ``scheme://`` URL is resolved through ``fsspec`` (``hdfs://``, ``s3://``,
  ``memory://`` …) when the corresponding backend is importable — tests use ``memory://`` as the
  in-process stand-in for the reference's ``MiniDFSCluster`` (`T/api/reader/ModelReaderSpec.scala:107-129`);
* the reader is a frozen, picklable dataclass so it can be shipped to worker processes like the
  reference's serializable case class.
"""

from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from urllib.parse import urlparse


class FsReader:
    """Mixin with the file-system access (`S/api/reader/FsReader.scala:32-49`)."""

    source_path: str

    @staticmethod
    def filesystem_for(path: str):
        """Return ``(kind, fs)`` for a path: ``("local", None)`` or ``("fsspec", fs)``."""
        parsed = urlparse(path)
        if parsed.scheme in ("", "file") or (len(parsed.scheme) == 1 and os.name == "nt"):
            return "local", None
        try:
            import fsspec  # noqa: F401
        except ImportError as e:  # pragma: no cover
            raise OSError(f"no file-system backend for {path!r} (fsspec not importable)") from e
        import fsspec

        return "fsspec", fsspec.filesystem(parsed.scheme)

    def read_bytes(self) -> bytes:
        path = self.source_path
        if path is None:
            raise FileNotFoundError("model path is None")
        kind, fs = self.filesystem_for(path)
        if kind == "local":
            local = urlparse(path).path if path.startswith("file://") else path
            with open(local, "rb") as fh:  # loan pattern: the handle is always closed
                data = fh.read()
        else:
            with fs.open(path, "rb") as fh:
                data = fh.read()
        from ..utils.faults import injector

        fi = injector()
        return fi.on_read(path, data) if fi.active else data

    def build_distributed_path(self) -> str:
        """Whole document as text (the reference's — oddly named — ``buildDistributedPath``)."""
        return self.read_bytes().decode("utf-8")

    buildDistributedPath = build_distributed_path  # noqa: N815

    def sha256(self) -> str:
        return hashlib.sha256(self.read_bytes()).hexdigest()


@dataclass(frozen=True)
class ModelReader(FsReader):
    source_path: str

    @property
    def sourcePath(self) -> str:  # noqa: N802
        return self.source_path
