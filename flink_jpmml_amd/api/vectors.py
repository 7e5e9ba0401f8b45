"""Input vectors: ``DenseVector`` and ``SparseVector`` (FlinkML ``Vector`` analogues used by the
reference API, `S/api/converter/VectorConverter.scala:58-86`).

Both are light wrappers over numpy arrays. Batches of vectors are packed into one
``[rows, size]`` float matrix with ``NaN`` for absent sparse entries by :func:`pack_vectors`
(host side) or the ``pack_csr`` HIP kernel (device side).
"""

from __future__ import annotations

from typing import Iterable, List, Sequence, Union

import numpy as np


class Vector:
    size: int

    def to_dense_array(self) -> np.ndarray:  # NaN for absent entries
        raise NotImplementedError


class DenseVector(Vector):
    __slots__ = ("data",)

    def __init__(self, *values):
        if len(values) == 1 and not np.isscalar(values[0]):
            data = np.asarray(values[0], dtype=np.float64)
        else:
            data = np.asarray(values, dtype=np.float64)
        self.data = data.reshape(-1)

    @property
    def size(self) -> int:
        return int(self.data.shape[0])

    def __getitem__(self, i: int) -> float:
        return float(self.data[i])

    def to_dense_array(self) -> np.ndarray:
        return self.data

    def __eq__(self, other: object) -> bool:
        return isinstance(other, DenseVector) and np.array_equal(self.data, other.data, equal_nan=True)

    def __hash__(self) -> int:
        return hash(self.data.tobytes())

    def __repr__(self) -> str:
        return f"DenseVector({', '.join(repr(float(x)) for x in self.data)})"


class SparseVector(Vector):
    __slots__ = ("_size", "indices", "data")

    def __init__(self, size: int, indices: Sequence[int], data: Sequence[float]):
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        val = np.asarray(data, dtype=np.float64).reshape(-1)
        if idx.shape != val.shape:
            raise ValueError("SparseVector: indices and data must have the same length")
        if idx.size and (idx.min() < 0 or idx.max() >= size):
            raise IndexError("SparseVector: index out of range")
        order = np.argsort(idx, kind="stable")
        self._size = int(size)
        self.indices = idx[order]
        self.data = val[order]

    @property
    def size(self) -> int:
        return self._size

    def __getitem__(self, i: int) -> float:
        pos = np.searchsorted(self.indices, i)
        if pos < self.indices.size and self.indices[pos] == i:
            return float(self.data[pos])
        return 0.0

    def to_dense_array(self) -> np.ndarray:
        out = np.full(self._size, np.nan)
        out[self.indices] = self.data
        return out

    def __eq__(self, other: object) -> bool:
        return (isinstance(other, SparseVector) and self._size == other._size
                and np.array_equal(self.indices, other.indices) and np.array_equal(self.data, other.data))

    def __hash__(self) -> int:
        return hash((self._size, self.indices.tobytes(), self.data.tobytes()))

    def __repr__(self) -> str:
        return f"SparseVector({self._size}, {self.indices.tolist()}, {self.data.tolist()})"


VectorLike = Union[Vector, Sequence[float], np.ndarray]


def as_vector(v: VectorLike) -> Vector:
    if isinstance(v, Vector):
        return v
    return DenseVector(np.asarray(v, dtype=np.float64))


def pack_vectors(vectors: Iterable[VectorLike], width: int) -> np.ndarray:
    """Pack dense/sparse vectors of size ``width`` into a ``[rows, width]`` float64 matrix with NaN
    for absent entries. Vectors of the wrong size must be filtered out beforehand."""
    vs: List[Vector] = [as_vector(v) for v in vectors]
    out = np.full((len(vs), width), np.nan)
    for i, v in enumerate(vs):
        if isinstance(v, SparseVector):
            out[i, v.indices] = v.data
        else:
            out[i, :] = v.data
    return out


def pack_vectors_masked(vectors: Iterable[VectorLike], width: int):
    """Like :func:`pack_vectors` but for vectors of any size: returns ``(X, absent, ok)`` where
    ``absent[i, j]`` marks entries a sparse vector does not store (the only positions the
    reference's ``replaceNaN`` fills, `S/api/PmmlModel.scala:143-152`; a NaN *stored* in a vector
    is kept as a PMML missing value) and ``ok[i]`` is False for vectors whose size is not
    ``width`` (their row is all-NaN; the per-record path fails their validation).

    Fast path: a batch of equal-width DenseVectors is one ``np.stack`` and returns ``ok=None``
    (every row conforms) and ``absent=None`` when no entry is NaN (nothing to tell apart); stored
    NaNs get an all-False mask so ``replace_nan`` leaves them missing, as per record."""
    vs = vectors if isinstance(vectors, list) else list(vectors)
    fp = _fastpath()
    if fp is not None and vs:
        X = np.empty((len(vs), width))
        if fp.pack_dense(vs, DenseVector, int(width), X) >= 0:
            return X, (np.zeros(X.shape, dtype=bool) if np.isnan(X).any() else None), None
    if vs and all(type(v) is DenseVector and len(v.data) == width for v in vs):
        X = np.concatenate([v.data for v in vs]).reshape(len(vs), width)
        return X, (np.zeros(X.shape, dtype=bool) if np.isnan(X).any() else None), None
    vs = [as_vector(v) for v in vs]
    n = len(vs)
    out = np.full((n, width), np.nan)
    absent = np.zeros((n, width), dtype=bool)
    ok = np.ones(n, dtype=bool)
    for i, v in enumerate(vs):
        if v.size != width:
            ok[i] = False
            continue
        if isinstance(v, SparseVector):
            absent[i, :] = True
            absent[i, v.indices] = False
            out[i, v.indices] = v.data
        else:
            out[i, :] = v.data
    return out, absent, ok


def _fastpath():
    from ..native import fastpath

    return fastpath()


def to_csr(vectors: Sequence[VectorLike], width: int):
    """CSR view ``(indptr int32, indices int32, values float32)`` of a vector batch — the input of the
    device-side ``pack_csr`` kernel (dense vectors contribute all their entries)."""
    indptr = np.zeros(len(vectors) + 1, dtype=np.int32)
    idx_parts, val_parts = [], []
    for i, v in enumerate(vectors):
        v = as_vector(v)
        if isinstance(v, SparseVector):
            idx_parts.append(v.indices.astype(np.int32))
            val_parts.append(v.data.astype(np.float32))
        else:
            idx_parts.append(np.arange(v.size, dtype=np.int32))
            val_parts.append(v.data.astype(np.float32))
        indptr[i + 1] = indptr[i] + idx_parts[-1].size
    idx = np.concatenate(idx_parts) if idx_parts else np.zeros(0, np.int32)
    val = np.concatenate(val_parts) if val_parts else np.zeros(0, np.float32)
    return indptr, idx, val
