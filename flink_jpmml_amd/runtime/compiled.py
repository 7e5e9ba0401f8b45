"""``CompiledPmml``: a parsed PMML document bound to its evaluator and (lazily) its device plan.

Load path (replaces `S/api/PmmlModel.scala:53-61`): text → :func:`parse_string` → IR →
:class:`FieldSchema` + family evaluator (float64 oracle) → on first GPU use
:func:`flink_jpmml_amd.runtime.plans.compile_plan` lowers it to device tensors.

Batch scoring contract (used by every streaming operator and the benchmark)::

    scores, valid = compiled.score_matrix(X)          # X: [rows, active_fields], NaN = missing

``scores`` is the reference's *target value as a double* (`S/api/pipeline/Pipeline.scala:93-98`),
``valid`` is False where the reference would return ``EmptyScore``.
"""

from __future__ import annotations

import logging
import threading
from typing import Any, Dict, List, Optional

import numpy as np

from ..api.exceptions import ModelLoadingException, PmmlParseError
from ..models import ModelResult, make_evaluator, result_scores
from ..pmml import ir
from ..pmml.fields import Columns, FieldSchema
from ..pmml.parser import parse_string
from ..pmml.validate import validate_literals

logger = logging.getLogger(__name__)


class CompiledPmml:
    def __init__(self, doc: ir.PMMLDocument, source: Optional[str] = None):
        self.doc = doc
        self.source = source
        self.schema = FieldSchema(doc)
        self.evaluator = make_evaluator(doc.model, self.schema)
        validate_literals(doc, self.schema)  # junk literals on numeric fields fail the load
        self.model = doc.model
        self.active_fields: List[str] = list(self.evaluator.active_fields)
        self.mining_fields: Dict[str, ir.MiningField] = dict(self.evaluator.mining_fields)
        self.target_fields: List[str] = list(self.evaluator.target_fields)
        self.output_fields: List[str] = [o.name for o in self.model.output]
        self._plans: Dict[str, Any] = {}
        self._lock = threading.Lock()

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_string(text, source: Optional[str] = None) -> "CompiledPmml":
        """From the document text (``str``) or its UTF-8 bytes."""
        return CompiledPmml(parse_string(text), source)

    @staticmethod
    def load(path: str) -> "CompiledPmml":
        from ..api.reader import ModelReader

        try:
            return CompiledPmml.from_string(ModelReader(path).read_bytes(), source=path)
        except (OSError, PmmlParseError, ValueError) as e:
            raise ModelLoadingException(str(e), e) from e

    @property
    def model_name(self) -> Optional[str]:
        return self.model.model_name

    @property
    def n_features(self) -> int:
        return len(self.active_fields)

    # ------------------------------------------------------------------ host oracle
    def columns(self, X: np.ndarray) -> Columns:
        X = np.asarray(X, dtype=np.float64)
        base = {name: X[:, j] for j, name in enumerate(self.active_fields)}
        cols = Columns(self.schema, X.shape[0], base)
        mindex = self.__dict__.get("_mindex")
        if mindex is None:
            mindex = self._mindex = {name: j for j, name in enumerate(self.active_fields)}
        cols.matrix, cols.mindex = X, mindex
        return cols

    def evaluate_prepared(self, X: np.ndarray) -> tuple:
        """Oracle over a *prepared* matrix. Returns ``(ModelResult, outputs dict)``."""
        cols = self.columns(X)
        res = self.evaluator.evaluate(cols)
        outs = self.evaluator.compute_outputs(cols, res) if self.model.output else {}
        return res, outs

    def prepare(self, X: np.ndarray, replace_nan: Optional[float] = None, absent: Optional[np.ndarray] = None) -> tuple:
        """MiningField preparation of a raw matrix. ``replace_nan`` fills the ``absent`` entries
        (entries a sparse vector does not store); without a mask every NaN counts as absent."""
        X = np.asarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[1] != self.n_features:
            raise ValueError(f"expected a [rows, {self.n_features}] matrix, got {X.shape}")
        if replace_nan is not None:
            X = np.where(np.isnan(X) if absent is None else absent, replace_nan, X)
        return self.schema.prepare_matrix(self.active_fields, X, self.mining_fields)

    def score_matrix_oracle(self, X: np.ndarray, replace_nan: Optional[float] = None,
                            absent: Optional[np.ndarray] = None) -> tuple:
        P, ok = self.prepare(X, replace_nan, absent)
        if not self.target_fields:
            # no named target: JPMML exposes only the synthetic null-named target, which the
            # reference drops (`S/api/pipeline/Pipeline.scala:79-85`) -> extraction fails
            return np.full(P.shape[0], np.nan), np.zeros(P.shape[0], dtype=bool)
        res, _ = self.evaluate_prepared(P)
        s, v = result_scores(res)
        v = v & ok
        return np.where(v, s, np.nan), v

    # ------------------------------------------------------------------ device
    def plan(self, device: Any = "cuda", **opts):
        """Lower to device tensors once per (device, options) and cache the plan."""
        from .plans import compile_plan

        key = f"{device}|{sorted(opts.items())}"
        with self._lock:
            p = self._plans.get(key)
            if p is None:
                p = compile_plan(self, device, **opts)
                self._plans[key] = p
            return p

    def score_matrix(self, X, replace_nan: Optional[float] = None, device: Any = None,
                     absent: Optional[np.ndarray] = None, **opts):
        """Batch scoring; ``device=None`` → host oracle, else the HIP plan on that device."""
        if device is None:
            return self.score_matrix_oracle(X, replace_nan, absent)
        return self.plan(device, **opts).score(X, replace_nan=replace_nan, absent=absent)

    def result(self, X: np.ndarray) -> ModelResult:
        P, _ = self.prepare(X)
        res, _ = self.evaluate_prepared(P)
        return res
