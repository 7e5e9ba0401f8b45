"""CSV records parsed on the GPU (``TextBatchSource(parse="device")``).

The reference's jobs consume text streams (`E/CheckpointEvaluate.scala:80-82`, a
``socketTextStream``; the examples' sources). Parsing text on the host caps one node at ~7 GB/s of
CSV — about 20 M records/s of 32 fields, 20x below what one MI355X scores. Here the host only
moves bytes:

    zero copy:       the file is mmapped and page-locked once (hipHostRegister, read-only); the
                     copy engines DMA each chunk straight out of the page cache. Without the
                     registration: reader threads pread the chunk into a pinned ring slot.
    copy streams:    chunk ──H2D──▶ HBM (two streams, alternating chunks)
    parse stream:    row_start_count + scan ─▶ (host: the row count, to size the output)
                     ─▶ row_start_write ─▶ parse_rows_lds (a workgroup's byte span staged in LDS,
                        one lane per record, exact fp32, coalesced tile stores)
                     ─▶ RecordBatch(X on the device, ready event) for the scoring operator

A record the GPU's decimal fast path does not settle (fp32 rounding midpoints, subnormals,
``inf`` spellings, > 19 digits, junk) is flagged; the host re-parses exactly those lines with the
native host parser and patches their rows, so every value is bit-identical to
:class:`flink_jpmml_amd.native.RecordParser`. Software pipeline: while chunk ``i`` is being read,
chunk ``i-1``'s rows are counted and parsed and chunk ``i-2`` is handed downstream, so the copy
engine and the parse kernels overlap the host reads.
"""

from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Optional, Sequence

import numpy as np

from ..api.batch import RecordBatch
from ..utils.metrics import METRICS

TILE = 4096  # bytes per row_start_count workgroup (textparse.hip TP_TILE)
MISSING_LEN = 16
MAX_MISSING = 8


def device_parse_supported(compiled, columns: Sequence[str], missing: Sequence[str]) -> Optional[str]:
    """``None`` when the GPU parser covers this model / header, else why not (the caller parses on
    the host)."""
    fields = list(compiled.active_fields)
    if any(compiled.schema.is_string(f) for f in fields):
        return "categorical (string) active fields need the host vocabularies"
    toks = [t for t in missing if t]
    if len(toks) > MAX_MISSING or any(len(t.encode()) >= MISSING_LEN for t in toks):
        return "missing-value tokens beyond the device table"
    absent = [f for f in fields if f not in list(columns)]
    if absent:
        return f"input columns lack active fields {absent}"
    return None


def _line_at(data: np.ndarray, start: int) -> bytes:
    """The line starting at ``start`` of a chunk that ends with a newline (newline included)."""
    w = 4096
    while True:
        seg = bytes(data[start: start + w])
        e = seg.find(b"\n")
        if e >= 0:
            return seg[: e + 1]
        w *= 4


HOST_REGISTER_READONLY = 0x08  # hipHostRegisterReadOnly: the device only reads the pages


class _MappedFile:
    """The whole file mapped read-only and page-locked for DMA: chunks then cross PCIe straight from
    the page cache — no host memcpy into a staging buffer, no reader threads. Registration faults
    every page in once; the mapping stays registered while the file is unchanged (same device,
    inode, size and mtime), so a job that re-reads its input pays it once."""

    def __init__(self, path: str, lib):
        import mmap

        st = os.stat(path)
        self.key = (st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns)
        self.lib = lib
        with open(path, "rb") as fh:
            self.mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
        self.data = np.frombuffer(self.mm, dtype=np.uint8)
        self.addr = int(self.data.ctypes.data)
        rc = lib.pmml_host_register(self.addr, len(self.data), HOST_REGISTER_READONLY)
        if rc != 0:
            self.data = None
            self.mm.close()
            raise OSError(f"hipHostRegister of {path} failed ({rc})")

    def release(self) -> None:
        if self.data is not None:
            self.lib.pmml_host_unregister(self.addr)
            self.data = None
            try:
                self.mm.close()
            except BufferError:  # a caller still holds a view; the mapping goes with it
                pass


_MAPPED: dict = {}  # path -> _MappedFile
_MAP_FAILED: set = set()  # keys whose registration failed (then positional reads)


def _mapped(path: str, lib) -> Optional[_MappedFile]:
    if not hasattr(lib, "pmml_host_register"):
        return None
    st = os.stat(path)
    key = (st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns)
    m = _MAPPED.get(path)
    if m is not None and m.key == key and m.data is not None:
        return m
    if m is not None:
        m.release()
        del _MAPPED[path]
    if key in _MAP_FAILED or st.st_size == 0:
        return None
    try:
        m = _MappedFile(path, lib)
    except (OSError, ValueError):
        _MAP_FAILED.add(key)
        METRICS.inc("ingest.device_text_register_failed")
        return None
    _MAPPED[path] = m
    return m


def release_mapped() -> None:
    """Unregister and unmap every cached file mapping."""
    for m in list(_MAPPED.values()):
        m.release()
    _MAPPED.clear()


class _Chunk:
    __slots__ = ("lo", "hi", "pinned", "n", "dev", "ev_h2d", "counts", "tot_h", "ev_cnt", "rows", "X", "starts",
                 "flag_h", "flagged", "ev_parse", "slot", "host")


class DeviceTextReader:
    """Reads one rank's byte range ``[lo, hi)`` of a CSV file and yields device RecordBatches."""

    def __init__(self, path: str, compiled, columns: Sequence[str], lo: int, hi: int, device, delimiter: str = ",",
                 missing: Sequence[str] = ("", "NA", "NaN", "nan", "?", "null", "NULL"),
                 chunk_bytes: int = 64 << 20, threads: int = 8, model_id: Optional[str] = None,
                 max_flagged: int = 1 << 16, zero_copy: bool = True, copy_streams: int = 2):
        import torch

        from ..ops import _lib

        self.path, self.compiled, self.columns = path, compiled, list(columns)
        self.lo, self.hi = int(lo), int(hi)
        self.device = torch.device(device)
        self.delim = delimiter.encode()[:1]
        self.missing = [t for t in missing if t]
        self.chunk_bytes = int(chunk_bytes)
        self.threads = max(1, int(threads))
        self.model_id = model_id
        self.max_flagged = int(max_flagged)
        self.zero_copy = bool(zero_copy)
        self.lib = _lib.load()
        fields = list(compiled.active_fields)
        pos = {f: j for j, f in enumerate(fields)}
        self.F = len(fields)
        self.colmap = torch.tensor([pos.get(c, -1) for c in self.columns], dtype=torch.int32, device=self.device)
        tab = np.zeros((MAX_MISSING, MISSING_LEN), dtype=np.uint8)
        for i, t in enumerate(self.missing):
            b = t.encode()
            tab[i, : len(b)] = np.frombuffer(b, dtype=np.uint8)
        self.missing_dev = torch.from_numpy(tab.reshape(-1)).to(self.device)
        # two copy streams, alternating chunks: both SDMA engines move bytes (one stream tops out
        # near 45 GB/s of the link, profiles/r4d)
        self.copies = [torch.cuda.Stream(self.device) for _ in range(max(1, int(copy_streams)))]
        self.parse = torch.cuda.Stream(self.device)
        self.host_parser = None
        self.bytes_read = 0
        self.rows_flagged = 0

    # ------------------------------------------------------------------ host side
    def _chunks(self) -> List[tuple]:
        """Chunk byte ranges ending just after a newline (the last one at ``hi``)."""
        out = []
        a = self.lo
        with open(self.path, "rb") as fh:
            while a < self.hi:
                b = min(self.hi, a + self.chunk_bytes)
                if b < self.hi:
                    fh.seek(b - 1)
                    b = b - 1 + len(fh.readline())  # through the next newline
                    b = min(b, self.hi)
                out.append((a, b))
                a = b
        return out

    def _read(self, fd: int, pool: ThreadPoolExecutor, lo: int, hi: int, dst) -> None:
        view = memoryview(dst.numpy()).cast("B")
        n = hi - lo
        step = max(1 << 20, -(-n // self.threads))

        def span(a: int) -> None:
            done, m = 0, min(step, n - a)
            while done < m:
                k = os.preadv(fd, [view[a + done: a + m]], lo + a + done)
                if k <= 0:
                    raise EOFError(f"{self.path}: short read at byte {lo + a + done}")
                done += k

        for f in [pool.submit(span, a) for a in range(0, n, step)]:
            f.result()

    # ------------------------------------------------------------------ pipeline stages
    def _submit_copy(self, c: _Chunk) -> None:
        import torch

        n = c.n
        cs = self.copies[c.slot % len(self.copies)]
        with torch.cuda.stream(cs):
            c.dev = torch.empty(n, dtype=torch.uint8, device=self.device)
            if c.pinned is not None:
                c.dev.copy_(c.pinned[:n], non_blocking=True)
            else:  # registered file mapping: DMA straight from the page cache
                m = c.hi - c.lo
                rc = self.lib.pmml_memcpy_async(c.dev.data_ptr(), int(c.host.ctypes.data), m, 1,
                                                cs.cuda_stream)  # hipMemcpyHostToDevice
                if rc != 0:
                    raise RuntimeError(f"H2D copy from the registered mapping failed ({rc})")
                if n > m:
                    c.dev[m:].fill_(10)  # the file's last line without a newline
            c.ev_h2d = torch.cuda.Event()
            c.ev_h2d.record(cs)
        tiles = -(-n // TILE)
        self.parse.wait_event(c.ev_h2d)
        with torch.cuda.stream(self.parse):
            c.counts = torch.empty(tiles + 1, dtype=torch.int32, device=self.device)
            rc = self.lib.pmml_text_rows_count(self.parse.cuda_stream, c.dev.data_ptr(), n, c.counts.data_ptr())
            if rc != 0:
                raise RuntimeError(f"text row count kernel failed ({rc})")
            c.tot_h = torch.empty(1, dtype=torch.int32, pin_memory=True)
            c.tot_h.copy_(c.counts[tiles:], non_blocking=True)
            c.ev_cnt = torch.cuda.Event()
            c.ev_cnt.record(self.parse)

    def _submit_parse(self, c: _Chunk) -> None:
        import torch

        from ..ops._lib import TextParseArgs

        c.ev_cnt.synchronize()
        c.rows = int(c.tot_h[0])
        with torch.cuda.stream(self.parse):
            c.starts = torch.empty(max(1, c.rows), dtype=torch.int64, device=self.device)
            c.X = torch.empty((c.rows, self.F), dtype=torch.float32, device=self.device)
            c.flagged = torch.empty(self.max_flagged + 1, dtype=torch.int32, device=self.device)
            c.flagged[-1:].zero_()
            rc = self.lib.pmml_text_rows_write(self.parse.cuda_stream, c.dev.data_ptr(), c.n, c.counts.data_ptr(),
                                               c.starts.data_ptr())
            if rc != 0:
                raise RuntimeError(f"text row index kernel failed ({rc})")
            a = TextParseArgs()
            a.buf, a.n_bytes, a.starts, a.n_rows = c.dev.data_ptr(), c.n, c.starts.data_ptr(), c.rows
            a.n_cols, a.colmap, a.F = len(self.columns), self.colmap.data_ptr(), self.F
            a.delim = self.delim
            a.n_missing, a.missing = len(self.missing), self.missing_dev.data_ptr()
            a.X = c.X.data_ptr()
            a.flagged, a.max_flagged = c.flagged.data_ptr(), self.max_flagged
            a.n_flagged = c.flagged[self.max_flagged:].data_ptr()
            import ctypes

            rc = self.lib.pmml_text_parse(self.parse.cuda_stream, ctypes.byref(a))
            if rc != 0:
                raise RuntimeError(f"text parse kernel failed ({rc})")
            c.flag_h = torch.empty(1, dtype=torch.int32, pin_memory=True)
            c.flag_h.copy_(c.flagged[self.max_flagged:], non_blocking=True)
            c.ev_parse = torch.cuda.Event()
            c.ev_parse.record(self.parse)
        c.dev.record_stream(self.parse)

    def _finish(self, c: _Chunk) -> RecordBatch:
        """Wait for the parse, patch the flagged records with the host parser."""
        import torch

        c.ev_parse.synchronize()
        k = int(c.flag_h[0])
        if k:
            self.rows_flagged += k
            METRICS.inc("ingest.device_text_flagged_rows", k)
            host = self._host_parser()
            data = c.pinned.numpy()[: c.n] if c.pinned is not None else c.host
            if c.n > len(data):
                data = np.concatenate([data, np.full(c.n - len(data), 10, np.uint8)])
            if k > self.max_flagged:  # pathological input: the whole chunk on the host parser
                m, _ = host.parse(bytes(data))
                with torch.cuda.stream(self.parse):
                    c.X.copy_(torch.from_numpy(m))
            else:
                rows = c.flagged[:k].cpu().numpy().astype(np.int64)
                starts = c.starts[torch.from_numpy(rows).to(self.device)].cpu().numpy()
                lines = [_line_at(data, st) for st in starts.tolist()]
                m, _ = host.parse(b"".join(lines))
                if len(m) != k:  # every flagged line is a non-empty record
                    raise RuntimeError(f"host re-parse of {k} flagged records returned {len(m)} rows")
                with torch.cuda.stream(self.parse):
                    c.X.index_copy_(0, torch.from_numpy(rows).to(self.device),
                                    torch.from_numpy(np.ascontiguousarray(m)).to(self.device))
            ev = torch.cuda.Event()
            ev.record(self.parse)
            c.ev_parse = ev
        c.X.record_stream(self.parse)
        return c

    def _host_parser(self):
        if self.host_parser is None:
            from .. import native

            self.host_parser = native.RecordParser(self.compiled, self.columns, delimiter=self.delim.decode(),
                                                   missing=[""] + self.missing, threads=self.threads)
        return self.host_parser

    # ------------------------------------------------------------------ iteration
    def __iter__(self) -> Iterator[RecordBatch]:
        import torch

        spans = self._chunks()
        if not spans:
            return
        mapped = _mapped(self.path, self.lib) if self.zero_copy else None
        self.zero_copy_active = mapped is not None
        ring: List = []
        ring_ev: List[Optional[object]] = [None] * 3
        fd = pool = None
        if mapped is None:
            cap = max(b - a for a, b in spans) + 1
            ring = [torch.empty(cap, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
            fd = os.open(self.path, os.O_RDONLY)
            pool = ThreadPoolExecutor(self.threads, thread_name_prefix="fja-text-read")
        row = 0
        stage_b: List[_Chunk] = []  # copied, counting
        stage_c: List[_Chunk] = []  # parsing
        try:
            for i in range(len(spans) + 2):
                if i < len(spans):
                    lo, hi = spans[i]
                    c = _Chunk()
                    c.slot = i % 3
                    n = hi - lo
                    if mapped is not None:
                        c.pinned, c.host = None, mapped.data[lo:hi]
                        if c.host[n - 1] != 10:  # the file's last line without a newline
                            n += 1
                    else:
                        if ring_ev[c.slot] is not None:
                            ring_ev[c.slot].synchronize()  # the H2D (and host patching) of its last use is over
                        c.pinned = ring[c.slot]
                        with METRICS.timer("ingest.device_text_read_ms"):
                            self._read(fd, pool, lo, hi, c.pinned)
                        if c.pinned[n - 1] != 10:  # the file's last line without a newline
                            c.pinned[n] = 10
                            n += 1
                    c.lo, c.hi, c.n = lo, hi, n
                    self.bytes_read += hi - lo
                    METRICS.inc("ingest.device_text_bytes", hi - lo)
                    self._submit_copy(c)
                    stage_b.append(c)
                if stage_b and (len(stage_b) > 1 or i >= len(spans)):
                    c = stage_b.pop(0)
                    with METRICS.timer("ingest.device_text_count_wait_ms"):
                        self._submit_parse(c)
                    stage_c.append(c)
                if stage_c and (len(stage_c) > 1 or i >= len(spans)):
                    with METRICS.timer("ingest.device_text_parse_wait_ms"):
                        c = self._finish(stage_c.pop(0))
                    ring_ev[c.slot] = c.ev_parse
                    if c.rows:
                        rb = RecordBatch(c.X, model_id=self.model_id, offset=row)
                        rb.ready = c.ev_parse
                        row += c.rows
                        yield rb
        finally:
            if pool is not None:
                pool.shutdown(wait=True)
                os.close(fd)
            torch.cuda.current_stream(self.device).wait_stream(self.parse)


__all__ = ["DeviceTextReader", "device_parse_supported", "release_mapped"]
