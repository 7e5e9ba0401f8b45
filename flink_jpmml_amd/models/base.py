"""Common machinery of the PMML model families.

Each family (clustering, tree, mining, regression, neural network, SVM) implements

* ``_evaluate(cols) -> ModelResult`` — the **float64 host oracle**: vectorised numpy evaluation
  of the PMML semantics over a whole batch. It replaces JPMML's per-record object-graph
  interpreter (`S/api/PmmlModel.scala:159-160`) as the semantic reference for every GPU kernel;
* ``compile_device()`` (in :mod:`flink_jpmml_amd.runtime.plans`) — lowering to device tensors
  scored by the hand-written HIP kernels.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from ..api.exceptions import EvaluationException, UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema, eval_expression


@dataclass
class ModelResult:
    """Batch evaluation result of one model element.

    ``value``: regression value, or predicted category *index* into ``categories``
    (classification), or 0-based cluster index (clustering). ``valid`` is False where no
    prediction exists (PMML null/missing prediction → ``EmptyScore``)."""

    kind: str
    value: np.ndarray
    valid: np.ndarray
    categories: Optional[List[str]] = None
    probs: Optional[np.ndarray] = None
    entity_ids: Optional[List[str]] = None
    affinity: Optional[np.ndarray] = None  # per-row affinity of the winning entity
    entity_affinities: Optional[np.ndarray] = None  # [n, K]
    extra: Dict[str, Any] = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(self.value.shape[0])

    def label_strings(self) -> List[Optional[str]]:
        out: List[Optional[str]] = []
        for v, ok in zip(self.value, self.valid):
            if not ok or math.isnan(v):
                out.append(None)
            elif self.kind == "classification":
                out.append(self.categories[int(v)])
            elif self.kind == "clustering":
                out.append(self.entity_ids[int(v)])
            else:
                out.append(None)
        return out


class ModelEvaluator:
    """Base class: schema bookkeeping, targets, outputs."""

    kind = "regression"

    def __init__(self, model: ir.Model, schema: FieldSchema):
        self.model = model
        self.schema = schema
        schema.register_model(model)
        self.active_fields: List[str] = [f.name for f in model.mining_schema.active]
        self.mining_fields: Dict[str, ir.MiningField] = {f.name: f for f in model.mining_schema.fields}
        tf = model.mining_schema.targets
        self.target_fields: List[str] = [f.name for f in tf]
        self.target_field: Optional[str] = self.target_fields[0] if self.target_fields else None
        self.target: Optional[ir.Target] = None
        for t in model.targets:
            if t.field is None or t.field == self.target_field:
                self.target = t
                break
        fn = model.function_name
        if fn == "classification":
            self.kind = "classification"
        elif fn == "clustering":
            self.kind = "clustering"
        elif fn in ("regression", "mixed", ""):
            self.kind = "regression" if fn != "" else self.kind

    # ------------------------------------------------------------------ API
    def evaluate(self, cols: Columns) -> ModelResult:
        c = cols.child(self.model.local_transformations) if self.model.local_transformations else cols
        res = self._evaluate(c)
        if res.kind == "regression":
            self._apply_regression_target(res)
        if c is not cols:
            # nested models expose their output fields to the enclosing context
            cols.data.update({k: v for k, v in c.data.items() if k not in cols.data})
        return res

    def _evaluate(self, cols: Columns) -> ModelResult:  # pragma: no cover - abstract
        raise NotImplementedError

    # ------------------------------------------------------------------ targets
    def _apply_regression_target(self, res: ModelResult) -> None:
        t = self.target
        if t is None:
            return
        v = res.value
        # JPMML TargetUtil order: clip to [min, max] first, then rescale, then castInteger
        if t.min is not None:
            v = np.maximum(v, t.min)
        if t.max is not None:
            v = np.minimum(v, t.max)
        if t.rescale_factor != 1.0 or t.rescale_constant != 0.0:
            v = v * t.rescale_factor + t.rescale_constant
        if t.cast_integer == "round":
            v = np.floor(v + 0.5)
        elif t.cast_integer == "ceiling":
            v = np.ceil(v)
        elif t.cast_integer == "floor":
            v = np.floor(v)
        # Targets/TargetValue defaultValue: used when the model produced no prediction
        if t.values and t.values[0].default_value is not None:
            dv = t.values[0].default_value
            v = np.where(res.valid, v, dv)
            res.valid = np.ones_like(res.valid)
        res.value = v

    def classification_categories(self) -> List[str]:
        """Target categories in declaration order: DataField values, else Targets' TargetValues."""
        tf = self.target_field
        cats: List[str] = []
        if tf is not None:
            df = self.schema.data_fields.get(tf)
            if df is not None:
                cats = list(df.values)
        if not cats and self.target is not None:
            cats = [tv.value for tv in self.target.values if tv.value is not None]
        return cats

    # ------------------------------------------------------------------ outputs
    def compute_outputs(self, cols: Columns, res: ModelResult) -> Dict[str, np.ndarray]:
        """Evaluate ``<Output>`` fields into encoded columns and publish them into ``cols``."""
        out: Dict[str, np.ndarray] = {}
        n = res.n
        for of in self.model.output:
            col = self._output_column(of, cols, res, n)
            cols.set(of.name, col)
            out[of.name] = col
        return out

    def _encode_label(self, name: str, labels: List[Optional[str]]) -> np.ndarray:
        col = np.full(len(labels), NAN)
        for i, lab in enumerate(labels):
            if lab is not None:
                col[i] = self.schema.lookup(name, lab)
        return col

    def _encode_result_labels(self, name: str, res: ModelResult) -> np.ndarray:
        """Vectorised ``_encode_label(name, res.label_strings())``: the field encoding of each of
        the K categories / entities is looked up once, then gathered by the winning index."""
        labels = res.categories if res.kind == "classification" else \
            res.entity_ids if res.kind == "clustering" else None
        if labels is None:
            return np.full(res.n, NAN)
        codes = np.array([self.schema.lookup(name, lab) if lab is not None else NAN for lab in labels] + [NAN])
        v = np.asarray(res.value, dtype=np.float64)
        ok = np.asarray(res.valid, dtype=bool) & ~np.isnan(v)
        idx = np.where(ok, np.nan_to_num(v, nan=0.0), len(labels)).astype(np.int64)
        return codes[idx]

    def _output_column(self, of: ir.OutputField, cols: Columns, res: ModelResult, n: int) -> np.ndarray:
        feat = of.feature
        if feat in ("predictedValue", "predictedDisplayValue"):
            if res.kind == "regression":
                return np.where(res.valid, res.value, NAN)
            return self._encode_result_labels(of.name, res)
        if feat == "probability":
            if res.probs is None or res.categories is None:
                raise UnsupportedFeatureException(f"output {of.name!r}: model has no probabilities")
            if of.value is None:
                idx = np.where(res.valid, res.value, 0).astype(np.int64)
                p = res.probs[np.arange(n), idx]
            else:
                if of.value not in res.categories:
                    return np.zeros(n)
                p = res.probs[:, res.categories.index(of.value)]
            return np.where(res.valid, p, NAN)
        if feat in ("entityId", "clusterId"):
            if res.kind == "clustering":
                if feat == "clusterId":
                    return np.where(res.valid, res.value + 1.0, NAN)
                return self._encode_result_labels(of.name, res)
            ents = res.extra.get("entity_labels")
            if ents is not None:
                return self._encode_label(of.name, ents)
            raise UnsupportedFeatureException(f"output feature {feat!r} not available for this model")
        if feat in ("affinity", "clusterAffinity", "entityAffinity"):
            if res.affinity is None:
                raise UnsupportedFeatureException(f"output feature {feat!r} not available for this model")
            if of.value is not None and res.entity_affinities is not None and res.entity_ids is not None:
                if of.value in res.entity_ids:
                    return res.entity_affinities[:, res.entity_ids.index(of.value)]
            return np.where(res.valid, res.affinity, NAN)
        if feat == "transformedValue":
            if of.expression is None:
                return np.where(res.valid, res.value, NAN) if res.kind == "regression" else np.full(n, NAN)
            return eval_expression(of.expression, cols, out_field=of.name)
        if feat == "decision":
            if of.expression is not None:
                return eval_expression(of.expression, cols, out_field=of.name)
        if feat in ("warning", "reasonCode", "ruleValue", "residual", "standardError", "confidence"):
            return np.full(n, NAN)
        raise UnsupportedFeatureException(f"output feature {feat!r} not supported")

    def decode_outputs(self, out: Dict[str, np.ndarray], row: int) -> Dict[str, Any]:
        return {k: self.schema.decode(k, float(v[row])) for k, v in out.items()}


def result_scores(res: ModelResult) -> tuple:
    """Reference target extraction on a batch: ``(score float64[n], valid bool[n])``.

    Regression → value; classification / clustering → the predicted label parsed as a double
    (`S/api/pipeline/Pipeline.scala:93-98`: a String target is ``toDouble``-ed)."""
    if res.kind == "regression":
        ok = res.valid & ~np.isnan(res.value)
        return np.where(ok, res.value, NAN), ok
    labels = res.categories if res.kind == "classification" else res.entity_ids
    table = np.array([_to_double(s) for s in (labels or [])], dtype=np.float64)
    score = np.full(res.n, NAN)
    ok = res.valid & ~np.isnan(res.value)
    if len(table):
        idx = np.where(ok, res.value, 0).astype(np.int64)
        score = np.where(ok, table[idx], NAN)
    ok = ok & ~np.isnan(score)
    return score, ok


def _to_double(s: Optional[str]) -> float:
    if s is None:
        return NAN
    try:
        return float(s)
    except ValueError:
        return NAN


def require(cond: bool, msg: str) -> None:
    if not cond:
        raise EvaluationException(msg)
