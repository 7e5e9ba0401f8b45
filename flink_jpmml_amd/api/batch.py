"""Columnar record batches and lazily materialised prediction batches — the DSL's fast path.

The reference scores one record at a time: ``flatMap(EvaluationFunction)`` calls
``f(event, model)`` and the UDF calls ``model.predict(vector)`` per record
(`S/package.scala:76-82,138-142`). That call pattern cannot feed a GPU. Here the same operators
also accept **RecordBatch** elements — ``[rows, active fields]`` float32 matrices, ideally in
pinned host memory — and the same UDF signature receives the whole batch:

    def udf(batch, model):                      # batch: RecordBatch, model: PmmlModel
        return batch.payload, model.predict(batch)   # -> PredictionBatch (async, on the GPU)

``PmmlModel.predict`` on a RecordBatch returns a :class:`PredictionBatch`: a future over device
scores that the kernel epilogue writes straight into pinned host memory. Nothing blocks until
someone reads ``.scores`` / ``.valid``, iterates, or indexes it; ``Prediction`` objects are only
built when a consumer asks for one (``batch[i]``, iteration, :meth:`PredictionBatch.to_list`).
``PredictionBatch[i] == model.predict(batch.vector(i))`` for every row — the per-record contract
of the reference holds row by row.
"""

from __future__ import annotations

import time
from typing import Any, Iterator, List, Optional, Sequence

import numpy as np

from ..domain.prediction import EMPTY_PREDICTION, Prediction, Score
from .vectors import DenseVector, SparseVector, Vector, as_vector


class RecordBatch:
    """``rows × n_features`` records in one column-major-free float32 matrix (NaN = missing).

    * ``X`` — numpy array or torch tensor (pinned host memory, or already on the device);
    * ``model_id`` — the model every row is scored with (dynamic serving, BaseEvent contract for
      batches), or ``model_ids`` — one id per row: a sequence of id strings, or dictionary-encoded
      as ``(codes, keys)`` (int codes per row — numpy or a pinned torch tensor — indexing the list
      of id strings ``keys``; the columnar form a dynamic-serving source should produce);
    * ``absent`` — optional bool mask of entries *absent* from sparse inputs: ``replace_nan``
      applies exactly there (a NaN *stored* in a vector stays a PMML missing value, as per record);
    * ``payload`` — optional per-row original events (for UDFs that return them);
    * ``offset`` — position of the first row in its source (checkpoint offsets, ordering).
    """

    __slots__ = ("X", "model_id", "_ids", "_codes", "_keys", "absent", "payload", "offset", "row_index", "created",
                 "_size_ok", "ready")

    def __init__(self, X: Any, model_id: Optional[str] = None, model_ids: Any = None,
                 absent: Optional[np.ndarray] = None, payload: Optional[Sequence[Any]] = None, offset: int = 0,
                 row_index: Optional[np.ndarray] = None):
        if getattr(X, "ndim", 2) != 2:
            raise ValueError(f"RecordBatch needs a [rows, features] matrix, got shape {tuple(X.shape)}")
        self.X = X
        self.model_id = model_id
        self._ids = self._codes = self._keys = None
        self.model_ids = model_ids
        self.absent = absent
        self.payload = payload
        self.offset = int(offset)
        self.row_index = row_index
        self.created = time.monotonic()
        self._size_ok: Optional[np.ndarray] = None
        # device-resident X produced on another stream: the event its consumers wait on (None: the
        # producer's current stream, e.g. a tensor built on the job thread)
        self.ready = None
        n = len(self)
        ids = self._codes if self._codes is not None else self._ids
        for name, col in (("model_ids", ids), ("absent", absent), ("payload", payload)):
            if col is not None and len(col) != n:
                raise ValueError(f"RecordBatch.{name} has {len(col)} rows, X has {n}")

    # ------------------------------------------------------------------ per-row model ids
    @property
    def model_ids(self) -> Optional[np.ndarray]:
        """One id string per row (object array; materialised from the codes if encoded)."""
        if self._ids is None and self._codes is not None:
            codes = self._codes.numpy() if hasattr(self._codes, "numpy") else np.asarray(self._codes)
            self._ids = np.asarray(self._keys, dtype=object)[codes.astype(np.int64, copy=False)]
        return self._ids

    @model_ids.setter
    def model_ids(self, value: Any) -> None:
        self._ids = self._codes = self._keys = None
        if value is None:
            return
        if isinstance(value, tuple) and len(value) == 2 and not isinstance(value[0], str):
            codes, keys = value
            self._codes, self._keys = codes, [str(k) for k in keys]
        else:
            self._ids = np.asarray(value, dtype=object)

    @property
    def has_model_ids(self) -> bool:
        return self._ids is not None or self._codes is not None

    def id_codes(self):
        """``(codes, keys)``: the per-row id column dictionary-encoded (first-appearance order when
        encoded here; the native encoder runs at ~300 M rows/s on repeated id objects)."""
        if self._codes is None and self._ids is not None:
            from ..native import fastpath

            fp = fastpath()
            ids = np.ascontiguousarray(self._ids)
            if fp is not None:
                codes, keys = fp.group_ids(ids)
            else:
                uniq, first, inv = np.unique(ids, return_index=True, return_inverse=True)
                order = np.argsort(first, kind="stable")
                rank = np.empty(len(order), dtype=np.int32)
                rank[order] = np.arange(len(order), dtype=np.int32)
                codes, keys = rank[inv].astype(np.int32), [str(u) for u in uniq[order]]
            self._codes, self._keys = codes, [str(k) for k in keys]
        return self._codes, self._keys

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_vectors(vectors: Sequence[Any], width: int, model_id: Optional[str] = None,
                     payload: Optional[Sequence[Any]] = None) -> "RecordBatch":
        """Pack Dense/Sparse vectors (wrong-size vectors become all-NaN rows flagged in ``absent``
        and are reported invalid by :meth:`size_ok`)."""
        from .vectors import pack_vectors_masked

        X, absent, ok = pack_vectors_masked(vectors, width)
        # float64 on the host (the oracle then matches per-record predict bit for bit); the device
        # path stages it as float32 like every other input
        if absent is not None and not absent.any() and not np.isnan(X).any():
            absent = None  # no NaN at all: "every NaN is absent" and "nothing absent" coincide
        b = RecordBatch(X, model_id=model_id, absent=absent, payload=payload)
        b._size_ok = ok if ok is not None and not ok.all() else None
        return b

    @staticmethod
    def pinned(n: int, n_features: int) -> "RecordBatch":
        """An uninitialised batch in pinned host memory (fill ``X`` in place, e.g. from the native
        ingest). Pageable memory on hosts without a GPU (nothing to DMA to)."""
        import torch

        return RecordBatch(torch.empty((n, n_features), dtype=torch.float32,
                                       pin_memory=torch.cuda.is_available()))

    def to_pinned(self) -> "RecordBatch":
        """This batch with ``X`` copied into pinned host memory (no-op if already pinned)."""
        import torch

        if isinstance(self.X, torch.Tensor) and (self.X.is_pinned() or self.X.is_cuda):
            return self
        src = torch.from_numpy(np.ascontiguousarray(self.X, dtype=np.float32))
        Xp = torch.empty(src.shape, dtype=torch.float32, pin_memory=True)
        Xp.copy_(src)
        return self._with(Xp)

    def _ids_arg(self, rows: Optional[np.ndarray] = None) -> Any:
        if self._codes is not None:
            c = self._codes
            if rows is not None:
                c = (c.numpy() if hasattr(c, "numpy") else np.asarray(c))[rows]
            return (c, self._keys)
        if self._ids is not None:
            return self._ids if rows is None else self._ids[rows]
        return None

    def _with(self, X: Any, rows: Optional[np.ndarray] = None) -> "RecordBatch":
        if rows is None:
            b = RecordBatch(X, self.model_id, self._ids_arg(), self.absent, self.payload, self.offset, self.row_index)
        else:
            b = RecordBatch(X, self.model_id, self._ids_arg(rows),
                            None if self.absent is None else self.absent[rows],
                            None if self.payload is None else [self.payload[i] for i in rows], self.offset,
                            rows if self.row_index is None else self.row_index[rows])
        ok = self._size_ok
        if ok is not None:
            b._size_ok = ok if rows is None else ok[rows]
        b.created = self.created
        b.ready = self.ready
        return b

    # ------------------------------------------------------------------ access
    def __len__(self) -> int:
        return int(self.X.shape[0])

    @property
    def n_features(self) -> int:
        return int(self.X.shape[1])

    def numpy(self) -> np.ndarray:
        X = self.X
        if hasattr(X, "detach"):
            X = X.detach().cpu().numpy()
        return np.asarray(X)

    def vector(self, i: int) -> Vector:
        """Row ``i`` as the vector the per-record API would have seen."""
        row = self.numpy()[i].astype(np.float64)
        if self.absent is not None and self.absent[i].any():
            keep = ~self.absent[i]
            return SparseVector(row.shape[0], np.nonzero(keep)[0], row[keep])
        return DenseVector(row)

    def __iter__(self) -> Iterator[Vector]:
        for i in range(len(self)):
            yield self.vector(i)

    def size_ok(self) -> Optional[np.ndarray]:
        """Per-row "vector had the model's width" flags (None = all rows conform)."""
        return self._size_ok

    def group_rows(self):
        """``(keys, perm, starts)``: the rows grouped by model id — ``perm[starts[k]:starts[k+1]]``
        are the rows (ascending) of id ``keys[k]``. Linear time: native dictionary encoding +
        counting sort (no per-id scans of the column)."""
        codes, keys = self.id_codes()
        c = codes.numpy() if hasattr(codes, "numpy") else np.asarray(codes)
        c = np.ascontiguousarray(c, dtype=np.int32)
        from ..native import fastpath

        fp = fastpath()
        if fp is not None:
            perm, counts = fp.counting_sort(c, len(keys))
        else:
            perm = np.argsort(c, kind="stable").astype(np.int32)
            counts = np.bincount(c, minlength=len(keys))
        starts = np.zeros(len(keys) + 1, dtype=np.int64)
        np.cumsum(counts, out=starts[1:])
        return keys, perm, starts

    def split_by_model(self) -> List["RecordBatch"]:
        """One sub-batch per distinct model id (first-appearance order, stable within an id);
        ``row_index`` of each sub-batch maps back to this batch's rows. Device-resident ``X`` is
        gathered on the device (``index_select``), host ``X`` on the host."""
        if not self.has_model_ids:
            return [self]
        keys, perm, starts = self.group_rows()
        out = []
        X = self.X
        dev = hasattr(X, "index_select") and getattr(X, "is_cuda", False)
        if dev:
            import torch

            perm_t = torch.from_numpy(perm.astype(np.int64)).to(X.device, non_blocking=False)
        else:
            X = self.numpy()
        for k, key in enumerate(keys):
            a, b = int(starts[k]), int(starts[k + 1])
            if a == b:
                continue
            rows = perm[a:b].astype(np.int64)
            Xk = X.index_select(0, perm_t[a:b]) if dev else X[rows]
            sub = self._with(Xk, rows)
            sub.model_id, sub.model_ids = str(key), None
            out.append(sub)
        return out

    @property
    def modelId(self) -> Optional[str]:  # noqa: N802 - BaseEvent-style alias
        return self.model_id

    def __repr__(self) -> str:
        mid = f", model_id={self.model_id!r}" if self.model_id else ""
        return f"RecordBatch(rows={len(self)}, features={self.n_features}{mid})"


class PredictionBatch:
    """Scores of one RecordBatch, possibly still being computed on the GPU.

    ``scores`` (float32, NaN where invalid) and ``valid`` (bool) are numpy views of pinned host
    buffers the kernel epilogue writes into; reading either waits for the device event. Row
    ``i`` materialises as ``Prediction(Score(scores[i]))`` or the shared
    ``Prediction(EmptyScore)`` — exactly what ``model.predict`` returns for that record.

    ``device_out`` optionally holds ``(score, valid)`` device mirrors (all-gather sinks);
    ``row_ok`` marks rows that passed the per-record size validation (others are EmptyScore)."""

    __slots__ = ("_n", "_scores", "_valid", "_done", "_owner", "_on_done", "_row_ok", "device_out", "submitted",
                 "completed", "__weakref__")

    def __init__(self, n: int, scores: Any = None, valid: Any = None, done: Any = None, owner: Any = None,
                 on_done: Any = None, device_out: Any = None, row_ok: Optional[np.ndarray] = None):
        self._n = int(n)
        self._scores = scores
        self._valid = valid
        self._done = done
        self._owner = owner  # keeps pinned / device buffers alive while the kernel may still write them
        self._on_done = on_done
        self._row_ok = row_ok
        self.device_out = device_out
        self.submitted = time.perf_counter()
        self.completed: Optional[float] = None
        if done is None:
            self._finish()

    # ------------------------------------------------------------------ completion
    @property
    def ready(self) -> bool:
        return self._done is None or bool(self._done.query())

    def _finish(self) -> None:
        s, v = self._scores, self._valid
        if hasattr(s, "numpy"):
            s = s.numpy()
        if hasattr(v, "numpy"):
            v = v.numpy()
        s = np.asarray(s)
        v = np.asarray(v)
        if v.dtype != np.bool_:
            v = v.view(np.bool_) if v.dtype == np.uint8 else v.astype(bool)
        ok = self._row_ok
        if ok is not None and not ok.all():
            v = v & ok
            s = np.where(ok, s, np.float32(np.nan)).astype(s.dtype, copy=False)
        self._scores, self._valid = s, v
        self.completed = time.perf_counter()

    def wait(self) -> "PredictionBatch":
        if self._done is not None:
            self._done.synchronize()
            self._done = None
            self._finish()
            cb, self._on_done = self._on_done, None
            if cb is not None:
                cb(self)
        return self

    def __del__(self):  # never let a pinned buffer go back to the allocator under a running kernel
        try:
            if self._done is not None:
                self._done.synchronize()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    # ------------------------------------------------------------------ columnar access
    @property
    def scores(self) -> np.ndarray:
        return self.wait()._scores

    @property
    def valid(self) -> np.ndarray:
        return self.wait()._valid

    def values(self, default: float = float("nan")) -> np.ndarray:
        """Vectorised ``prediction.value.getOrElse(default)`` (float64)."""
        return np.where(self.valid, self.scores.astype(np.float64), default)

    get_or_else = values

    # ------------------------------------------------------------------ per-record access (lazy)
    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if self.valid[i]:
            return Prediction(Score(float(self.scores[i])))
        return EMPTY_PREDICTION

    def __iter__(self) -> Iterator[Prediction]:
        s, v = self.scores, self.valid
        for i in range(self._n):
            yield Prediction(Score(float(s[i]))) if v[i] else EMPTY_PREDICTION

    def to_list(self) -> List[Prediction]:
        return self.predictions()

    def predictions(self) -> List[Prediction]:
        """Every row as a :class:`Prediction` (one vectorised pass; the per-record streams'
        output path)."""
        valid = self.valid
        from ..native import fastpath

        fp = fastpath()
        if fp is not None:
            s = np.ascontiguousarray(self.scores, dtype=np.float32)
            out = fp.make_predictions(s, np.ascontiguousarray(valid), Prediction, Score, EMPTY_PREDICTION)
            if out is not None:
                return out
        out = list(map(Prediction, map(Score, self.scores.tolist())))
        if not valid.all():
            for i in np.flatnonzero(~valid).tolist():
                out[i] = EMPTY_PREDICTION
        return out

    def empty_count(self) -> int:
        return int(self._n - np.count_nonzero(self.valid))

    def __eq__(self, other: object) -> bool:
        if isinstance(other, PredictionBatch):
            return len(self) == len(other) and self.to_list() == other.to_list()
        if isinstance(other, (list, tuple)):
            return self.to_list() == list(other)
        return NotImplemented

    __hash__ = None  # type: ignore[assignment]

    def __repr__(self) -> str:
        state = "ready" if self.ready else "in flight"
        return f"PredictionBatch(rows={self._n}, {state})"

    def __reduce__(self):  # pickles as its (completed) arrays: checkpoint / all_gather_object safe
        return (PredictionBatch.from_arrays, (np.array(self.scores), np.array(self.valid)))

    # ------------------------------------------------------------------ construction helpers
    @staticmethod
    def from_arrays(scores: Any, valid: Any) -> "PredictionBatch":
        s = np.asarray(scores, dtype=np.float32)
        v = np.asarray(valid, dtype=bool)
        return PredictionBatch(len(s), s, v)

    @staticmethod
    def empty(n: int) -> "PredictionBatch":
        return PredictionBatch(n, np.full(n, np.nan, dtype=np.float32), np.zeros(n, dtype=bool))

    @staticmethod
    def concat(parts: Sequence["PredictionBatch"]) -> "PredictionBatch":
        if not parts:
            return PredictionBatch.empty(0)
        return PredictionBatch.from_arrays(np.concatenate([p.scores for p in parts]),
                                           np.concatenate([p.valid for p in parts]))

    def masked(self, ok: Optional[np.ndarray]) -> "PredictionBatch":
        """This batch with rows where ``ok`` is False forced to EmptyScore (validation failures)."""
        if ok is None or ok.all():
            return self
        return PredictionBatch.from_arrays(np.where(ok, self.scores, np.nan), self.valid & ok)


def as_record_batch(x: Any, width: Optional[int] = None) -> Optional[RecordBatch]:
    """``x`` as a RecordBatch if it is batch-shaped (RecordBatch, 2-D array/tensor), else None."""
    if isinstance(x, RecordBatch):
        return x
    if isinstance(x, np.ndarray) and x.ndim == 2:
        return RecordBatch(x)
    if hasattr(x, "dim") and callable(getattr(x, "dim")) and x.dim() == 2:
        return RecordBatch(x)
    return None


__all__ = ["PredictionBatch", "RecordBatch", "as_record_batch", "as_vector"]
