"""Zero-parse columnar ingest: raw fp32 record frames from files or sockets.

Text ingest costs ~300 bytes and a float parse per field; one MI355X scores 400+ M records/s, so a
stream that must feed it needs records that are already in the engine's layout. This module
defines a minimal binary framing of the ``[rows, n_features]`` fp32 row-major matrix the kernels
read and two sources for it (the reference's source side is Flink's, `S/package.scala:76-82`;
SURVEY §7.4 item 4):

* :class:`BinaryBatchSource` — a file: a 32-byte header (:data:`MAGIC`, version, n_features,
  n_rows) then the rows. Each batch is read straight from the page cache into a **pinned**
  buffer by a small thread pool of positional reads (``os.preadv`` into slices of the pinned
  buffer; no parse, the GIL is released) while the previous batch is being scored. Reads rather
  than a memory map: copying out of an mmap takes one minor page fault per 4 KiB source page,
  which capped the round-3 mmap source at ~27 GB/s (211.8 M rec/s, `profiles/r3ab/`), about half
  the PCIe rate. Under torchrun every rank reads only its own contiguous row range (rank-local
  split, F3).
* :class:`SocketBinarySource` — a TCP stream of frames (16-byte frame header: magic, n_rows,
  n_features, flags; then the payload) received with ``recv_into`` straight into pinned memory.

:func:`write_binary` / :func:`send_binary` produce the formats (``bench.py --source binary``,
tests).
"""

from __future__ import annotations

import os
import socket
import struct
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, Optional

import numpy as np

from ..api.batch import RecordBatch
from .functions import SourceFunction

MAGIC = b"FJAB"
VERSION = 1
FILE_HEADER = struct.Struct("<4sIIQQI")  # magic, version, n_features, n_rows, data offset, reserved
FRAME_MAGIC = 0x464A4146  # "FAJF"
FRAME_HEADER = struct.Struct("<IIII")   # magic, n_rows, n_features, flags (bit 0: end of stream)


def _pinned(rows: int, F: int):
    import torch

    return torch.empty((rows, F), dtype=torch.float32, pin_memory=torch.cuda.is_available())


def write_binary(path: str, X: np.ndarray) -> str:
    """Write ``X`` ([rows, F], cast to fp32) as a binary record file."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    rows, F = X.shape
    with open(path, "wb") as fh:
        fh.write(FILE_HEADER.pack(MAGIC, VERSION, F, rows, 64, 0).ljust(64, b"\0"))
        X.tofile(fh)
    return path


def read_header(path: str):
    with open(path, "rb") as fh:
        head = fh.read(FILE_HEADER.size)
    magic, version, F, rows, off, _ = FILE_HEADER.unpack(head)
    if magic != MAGIC or version != VERSION:
        raise ValueError(f"{path}: not a flink_jpmml_amd binary record file")
    return int(F), int(rows), int(off)


class BinaryBatchSource(SourceFunction):
    """Memory-mapped binary record file → pinned RecordBatches (see module docstring).

    ``threads`` parallel memcpy workers; ``prefetch`` batches copied ahead of the consumer.
    ``repeat`` replays the file (synthetic long streams)."""

    chunkable = False

    def __init__(self, path: str, batch_rows: int = 1 << 20, threads: int = 4, prefetch: int = 2,
                 repeat: int = 1, model_id: Optional[str] = None):
        self.path = path
        self.batch_rows = int(batch_rows)
        self.threads = max(1, int(threads))
        self.prefetch = max(1, int(prefetch))
        self.repeat = int(repeat)
        self.model_id = model_id
        self._rank, self._world = 0, 1
        self.bytes_read = 0

    def open_subtask(self, rank: int, world: int) -> None:
        self._rank, self._world = int(rank), int(world)

    def row_range(self, rows: int):
        lo = rows * self._rank // self._world
        hi = rows * (self._rank + 1) // self._world
        return lo, hi

    def iterate(self) -> Iterator[RecordBatch]:
        from ..utils.metrics import METRICS

        F, rows, off = read_header(self.path)
        fd = os.open(self.path, os.O_RDONLY)
        lo, hi = self.row_range(rows)
        B = self.batch_rows
        pool = ThreadPoolExecutor(self.threads, thread_name_prefix="fja-binary-copy")
        orch = ThreadPoolExecutor(self.prefetch, thread_name_prefix="fja-binary-batch")
        rb = F * 4
        try:
            os.posix_fadvise(fd, off + lo * rb, (hi - lo) * rb, os.POSIX_FADV_SEQUENTIAL)
        except (AttributeError, OSError):
            pass

        def read_span(view: memoryview, pos: int) -> None:
            done = 0
            while done < len(view):
                n = os.preadv(fd, [view[done:]], pos + done)
                if n <= 0:
                    raise EOFError(f"{self.path}: short read at byte {pos + done}")
                done += n

        def fill(s: int, e: int):
            buf = _pinned(e - s, F)
            dst = memoryview(buf.numpy()).cast("B")
            step = max(1, -(-(e - s) // self.threads))
            futs = [pool.submit(read_span, dst[(a - s) * rb:(min(e, a + step) - s) * rb], off + a * rb)
                    for a in range(s, e, step)]
            for f in futs:
                f.result()
            return buf

        spans = [(r, s, min(hi, s + B)) for r in range(self.repeat) for s in range(lo, hi, B)]
        ahead = []
        try:
            k = 0
            while k < len(spans) or ahead:
                while k < len(spans) and len(ahead) < self.prefetch:
                    r, s, e = spans[k]
                    ahead.append((r, s, e, orch.submit(fill, s, e)))
                    k += 1
                r, s, e, fut = ahead.pop(0)
                buf = fut.result()
                n = (e - s) * F * 4
                self.bytes_read += n
                METRICS.inc("ingest.binary_bytes", n)
                yield RecordBatch(buf, model_id=self.model_id, offset=r * rows + s)
        finally:
            orch.shutdown(wait=True)
            pool.shutdown(wait=True)
            os.close(fd)


def send_binary(sock: socket.socket, X: np.ndarray, end: bool = False) -> None:
    """Send one frame of records (``end=True`` closes the stream logically)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    rows, F = X.shape if X.size else (0, X.shape[1] if X.ndim == 2 else 0)
    sock.sendall(FRAME_HEADER.pack(FRAME_MAGIC, rows, F, 1 if end else 0))
    if rows:
        sock.sendall(memoryview(X).cast("B"))


class SocketBinarySource(SourceFunction):
    """TCP stream of binary record frames, each received straight into a pinned RecordBatch."""

    live = True

    def __init__(self, host: str, port: int, connect_timeout_s: float = 10.0, model_id: Optional[str] = None):
        self.host, self.port = host, int(port)
        self.connect_timeout_s = float(connect_timeout_s)
        self.model_id = model_id
        self._sock: Optional[socket.socket] = None
        self._running = True

    def cancel(self) -> None:
        self._running = False
        if self._sock is not None:
            try:
                self._sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass

    def _recv_exact(self, s: socket.socket, view: memoryview) -> bool:
        got = 0
        while got < len(view):
            n = s.recv_into(view[got:])
            if n == 0:
                return False
            got += n
        return True

    def iterate(self) -> Iterator[RecordBatch]:
        s = socket.create_connection((self.host, self.port), timeout=self.connect_timeout_s)
        s.settimeout(None)
        self._sock = s
        row = 0
        try:
            head = bytearray(FRAME_HEADER.size)
            while self._running:
                if not self._recv_exact(s, memoryview(head)):
                    return
                magic, rows, F, flags = FRAME_HEADER.unpack(head)
                if magic != FRAME_MAGIC:
                    raise ValueError("binary record stream: bad frame magic")
                if rows:
                    buf = _pinned(rows, F)
                    if not self._recv_exact(s, memoryview(buf.numpy()).cast("B")):
                        return
                    yield RecordBatch(buf, model_id=self.model_id, offset=row)
                    row += rows
                if flags & 1:
                    return
        finally:
            self._sock = None
            s.close()


__all__ = ["BinaryBatchSource", "FILE_HEADER", "MAGIC", "SocketBinarySource", "read_header", "send_binary",
           "write_binary"]
