"""``Vector`` → ``PmmlInput`` (``dict[str, Any]``) keyed by the model's active fields in
MiningSchema order.

Reference: `S/api/converter/VectorConverter.scala:31-103`.

* dense: ``zip(keys, data)`` — a short vector yields a *partial* map (the validation step normally
  rejects it first);
* sparse: only the present entries are mapped; absent entries are **absent keys**, not NaN, so
  PMML missing-value handling (or ``replace_nan``) applies to them.

Unlike the reference's O(size·nnz) densification (`:100-103`) this is O(nnz).
"""

from __future__ import annotations

from typing import Any, Dict, List

from .evaluator import Evaluator
from .vectors import DenseVector, SparseVector, Vector, as_vector

PmmlInput = Dict[str, Any]


def active_keys(evaluator: Evaluator) -> List[str]:
    return list(evaluator.model.active_fields)


def dense_to_map(vec: DenseVector, evaluator: Evaluator) -> PmmlInput:
    keys = active_keys(evaluator)
    return {k: float(v) for k, v in zip(keys, vec.data)}


def sparse_to_map(vec: SparseVector, evaluator: Evaluator) -> PmmlInput:
    keys = active_keys(evaluator)
    out: PmmlInput = {}
    for i, v in zip(vec.indices.tolist(), vec.data.tolist()):
        if i < len(keys):
            out[keys[i]] = float(v)
    return out


def vector_conversion(vec: Vector, evaluator: Evaluator) -> PmmlInput:
    vec = as_vector(vec)
    if isinstance(vec, SparseVector):
        return sparse_to_map(vec, evaluator)
    return dense_to_map(vec, evaluator)


# Scala-style aliases
denseVector2Map = dense_to_map  # noqa: N816
sparseVector2Map = sparse_to_map  # noqa: N816
vectorConversion = vector_conversion  # noqa: N816
