"""Native host runtime pieces (C++17, built with g++).

* ``_ingest.so`` (ctypes) — :class:`RecordParser` turns delimited text records into the engine's
  ``[rows, active fields]`` fp32 matrix on all cores (``csrc/ingest.cpp``), writing straight into a
  caller-provided (pinned) buffer — the host-ingest stage in front of the H2D copy. Categorical
  tokens are encoded with the model's PMML vocabularies (the same codes the float64 oracle uses),
  missing tokens become NaN.
* ``_fastpath`` (CPython extension, ``csrc/fastpath.cpp``) — the per-record stream path's object
  traffic: DenseVector lists → matrix, scored arrays → ``Prediction`` objects (:func:`fastpath`).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "ingest.cpp")
LIB_PATH = os.path.join(HERE, "_ingest.so")

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


class NativeBuildError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= os.path.getmtime(SRC):
        return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-fvisibility=hidden", SRC, "-o", tmp]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise NativeBuildError(r.stdout.decode(errors="replace"))
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


FAST_SRC = os.path.join(HERE, "csrc", "fastpath.cpp")
FAST_SRCS = [FAST_SRC, os.path.join(HERE, "csrc", "pmml_scan.cpp"), os.path.join(HERE, "csrc", "tree_walk.cpp"),
             os.path.join(HERE, "csrc", "nn_host.cpp")]
_fast = None


def _fast_path() -> str:
    import sysconfig

    return os.path.join(HERE, "_fastpath" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def build_fastpath(force: bool = False) -> str:
    """Compile the CPython fast-path extension in-tree (g++, Python + NumPy headers)."""
    import sysconfig

    out = _fast_path()
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(s) for s in FAST_SRCS):
        return out
    tmp = out + ".tmp"
    # -ffp-contract=off: the oracle's sums round every product and every partial sum (no FMA)
    cmd = ["g++", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-pthread", "-Wall", "-fvisibility=hidden",
           "-I" + sysconfig.get_paths()["include"], "-I" + np.get_include(), *FAST_SRCS, "-o", tmp]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise NativeBuildError(r.stdout.decode(errors="replace"))
    os.replace(tmp, out)
    return out


def fastpath():
    """The ``_fastpath`` extension module (built on first use; ``None`` if it cannot be built, the
    callers then use their pure-Python paths)."""
    global _fast
    if _fast is None:
        with _lock:
            if _fast is None:
                try:
                    import importlib.util

                    path = build_fastpath()
                    spec = importlib.util.spec_from_file_location("flink_jpmml_amd.native._fastpath", path)
                    mod = importlib.util.module_from_spec(spec)
                    spec.loader.exec_module(mod)
                    _fast = mod
                except Exception:  # noqa: BLE001 - pure-Python fallback keeps results identical
                    _fast = False
    return _fast or None


def load() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            build()
            lib = ctypes.CDLL(LIB_PATH)
            lib.ingest_vocab_new.restype = ctypes.c_void_p
            lib.ingest_vocab_new.argtypes = [ctypes.c_int]
            lib.ingest_vocab_free.argtypes = [ctypes.c_void_p]
            lib.ingest_vocab_add.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                             ctypes.c_float]
            lib.ingest_parse.restype = ctypes.c_longlong
            lib.ingest_parse.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
            _lib = lib
        return _lib


DEFAULT_MISSING = ("", "NA", "NaN", "nan", "?", "null", "NULL")


class RecordParser:
    """Parse delimited records whose columns are ``columns`` (e.g. the CSV header) into the
    model's active-field matrix. Columns the model does not use are skipped."""

    def __init__(self, compiled, columns: Sequence[str], delimiter: str = ",",
                 missing: Iterable[str] = DEFAULT_MISSING, threads: int = 0):
        self.lib = load()
        self.fields: List[str] = list(compiled.active_fields)
        pos = {f: j for j, f in enumerate(self.fields)}
        self.columns = list(columns)
        absent = [f for f in self.fields if f not in self.columns]
        if absent:
            raise ValueError(f"input columns lack active fields {absent}")
        self.target = np.array([pos.get(c, -1) for c in self.columns], dtype=np.int32)
        schema = compiled.schema
        self.kind = np.array([1 if schema.is_string(f) else 0 for f in self.fields], dtype=np.int32)
        self.vocab = self.lib.ingest_vocab_new(len(self.fields))
        for j, f in enumerate(self.fields):
            if self.kind[j]:
                for code, v in enumerate(schema.values.get(f, [])):
                    b = v.encode()
                    self.lib.ingest_vocab_add(self.vocab, j, b, len(b), float(code))
        self.delim = delimiter.encode()[:1]
        toks = list(missing)
        self.missing = b"".join(t.encode() + b"\0" for t in toks)
        self.n_missing = len(toks)
        self.threads = threads or max(1, min(16, os.cpu_count() or 1))
        self.bad_tokens = 0

    def __del__(self):
        v = getattr(self, "vocab", None)
        if v:
            self.lib.ingest_vocab_free(v)
            self.vocab = None

    def parse(self, data: Any, out: Optional[np.ndarray] = None, max_rows: Optional[int] = None,
              length: Optional[int] = None) -> Tuple[np.ndarray, int]:
        """Parse the complete lines of ``data`` (``bytes``, or a ``bytearray`` whose first
        ``length`` bytes are parsed in place — no copy). Returns ``(rows view of out, bytes
        consumed)``; ``out`` (float32 ``[cap, fields]``, e.g. a pinned tensor's numpy view) is
        allocated if omitted."""
        F = len(self.fields)
        if isinstance(data, bytearray):
            n_bytes = len(data) if length is None else int(length)
            if n_bytes > len(data):
                raise ValueError("length exceeds the buffer")
            if out is None:
                data = bytes(data[:n_bytes])  # sizing pass below needs the line count
            else:
                view = (ctypes.c_char * max(1, len(data))).from_buffer(data)  # exported while parsing
                return self._parse_ptr(ctypes.addressof(view), n_bytes, out, max_rows)
        elif length is not None:
            data = data[:length]
        if out is None:
            cap = max_rows if max_rows is not None else data.count(b"\n") + 1
            out = np.empty((cap, F), dtype=np.float32)
        if out.dtype != np.float32 or not out.flags.c_contiguous or out.shape[1] != F:
            raise ValueError(f"out must be a C-contiguous float32 [rows, {F}] array")
        return self._parse_ptr(data, len(data), out, max_rows)

    def parse_address(self, addr: int, n_bytes: int, out: np.ndarray, max_rows: Optional[int] = None
                      ) -> Tuple[np.ndarray, int]:
        """:meth:`parse` over ``n_bytes`` of host memory at ``addr`` (e.g. a memory-mapped file:
        parsed where it lies, no copy). The memory must stay valid for the call."""
        return self._parse_ptr(ctypes.c_void_p(int(addr)), int(n_bytes), out, max_rows)

    def _parse_ptr(self, data: Any, n_bytes: int, out: np.ndarray, max_rows: Optional[int]) -> Tuple[np.ndarray, int]:
        F = len(self.fields)
        if out.dtype != np.float32 or not out.flags.c_contiguous or out.shape[1] != F:
            raise ValueError(f"out must be a C-contiguous float32 [rows, {F}] array")
        cap = out.shape[0] if max_rows is None else min(max_rows, out.shape[0])
        consumed, bad = ctypes.c_size_t(0), ctypes.c_size_t(0)
        if n_bytes == 0 or cap == 0:
            return out[:0], 0
        n = self.lib.ingest_parse(data, n_bytes, self.delim, len(self.columns), self.target.ctypes.data, F,
                                  self.kind.ctypes.data, self.missing, self.n_missing, self.vocab,
                                  out.ctypes.data, cap, self.threads, ctypes.byref(consumed), ctypes.byref(bad))
        if n < 0:
            raise ValueError(f"ingest_parse failed with code {n}")
        self.bad_tokens += bad.value
        return out[:n], consumed.value

    def parse_file(self, path: str, chunk_bytes: int = 64 << 20):
        """Yield ``[rows, fields]`` batches of a delimited file (header line skipped if it
        matches ``columns``)."""
        with open(path, "rb") as fh:
            rest = b""
            first = True
            while True:
                blk = fh.read(chunk_bytes)
                data = rest + blk
                if first:
                    first = False
                    nl = data.find(b"\n")
                    head = data[:nl].decode(errors="replace").strip().split(self.delim.decode())
                    if [h.strip().strip('"') for h in head] == self.columns:
                        data = data[nl + 1:]
                if not blk:
                    if data and not data.endswith(b"\n"):
                        data += b"\n"
                    if data:
                        m, _ = self.parse(data)
                        if len(m):
                            yield m
                    return
                m, used = self.parse(data)
                rest = data[used:]
                if len(m):
                    yield m


def parse_records(compiled, text: bytes, columns: Sequence[str], **kw) -> np.ndarray:
    """One-shot convenience: delimited ``text`` -> ``[rows, active fields]`` float32."""
    m, _ = RecordParser(compiled, columns, **kw).parse(text if text.endswith(b"\n") else text + b"\n")
    return m


__all__ = ["RecordParser", "parse_records", "build", "load"]
