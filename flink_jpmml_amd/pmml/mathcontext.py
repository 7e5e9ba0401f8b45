"""``x-mathContext="float"``: models whose arithmetic is single precision.

JPMML converters for float-native learners (jpmml-xgboost, jpmml-lightgbm) mark their models
``x-mathContext="float"``: split thresholds, leaf scores and coefficients are float32 values and the
evaluator computes in float32 (the reference evaluates through JPMML: `S/api/PmmlModel.scala:159-160`).
Under a double evaluator such a model differs from the trainer wherever a threshold like ``0.1`` is
not float-representable (``x <= 0.1`` is TRUE in float for ``x = 0.1f``, FALSE in double) and in the
last bits of long sums.

:func:`apply_math_context` runs once per parsed document. For every model in float context (the
attribute is inherited by nested segment models unless they say ``double``) it rounds the numeric
literals the model computes with to float32 — ``SimplePredicate`` values on continuous fields,
regression tree scores, segment weights, regression coefficients — and records
``Model.math_context = "float"``. The oracle evaluators then accumulate in float32 where the
context says so (segment sums in segment order, regression tables in term order); the device
kernels compute in fp32 already, and with float32 literals their split decisions match the oracle
exactly. Parity unpinned (no JPMML here): follows the converters' documented intent.
"""

from __future__ import annotations

from typing import Dict, Iterable, Optional

import numpy as np

from . import ir


def _f32_str(v: float) -> str:
    return repr(float(np.float32(v)))


def _round_value(s: Optional[str]) -> Optional[str]:
    """A numeric literal rounded to float32 (unchanged if not numeric or already representable)."""
    if s is None:
        return s
    try:
        v = float(s)
    except ValueError:
        return s
    if not np.isfinite(v) or float(np.float32(v)) == v:
        return s
    return _f32_str(v)


def _continuous(fields: Dict[str, str], name: Optional[str]) -> bool:
    return fields.get(name, "continuous") == "continuous"


def _round_predicate(p, fields: Dict[str, str]):
    if isinstance(p, ir.SimplePredicate):
        if p.value is not None and _continuous(fields, p.field):
            p.value = _round_value(p.value)
    elif isinstance(p, ir.CompoundPredicate):
        for q in p.predicates:
            _round_predicate(q, fields)


def _round_flat(ft, fields: Dict[str, str], regression: bool) -> None:
    from .flat import P_SIMPLE

    a = ft.a
    strings = ft.strings
    if not isinstance(strings, list):
        strings = list(strings)
        ft.strings = strings
    index: Dict[str, int] = {}

    def intern(s: str) -> int:
        k = index.get(s)
        if k is None:
            k = len(strings)
            strings.append(s)
            index[s] = k
        return k

    kind, pf, vd = a["pred_kind"], a["pred_field"], a["pred_value_d"]
    cont = np.zeros(len(strings) + 1, dtype=bool)
    for k in np.unique(pf[kind == P_SIMPLE]).tolist():
        cont[k] = _continuous(fields, strings[k])
    m = (kind == P_SIMPLE) & np.isfinite(vd)
    m &= cont[np.where(m, pf, len(cont) - 1)]
    r = vd.astype(np.float32).astype(np.float64)
    m &= r != vd
    if m.any():
        vs = a["pred_value_s"].copy()
        for k in np.nonzero(m)[0].tolist():
            vs[k] = intern(_f32_str(vd[k]))
        a["pred_value_s"] = vs
        a["pred_value_d"] = np.where(m, r, vd)
    if regression and "score_d" in a:
        sd = a["score_d"]
        rs = sd.astype(np.float32).astype(np.float64)
        ms = np.isfinite(sd) & (rs != sd)
        if ms.any():
            ss = a["score_s"].copy()
            for k in np.nonzero(ms)[0].tolist():
                ss[k] = intern(_f32_str(sd[k]))
            a["score_s"] = ss
            a["score_d"] = np.where(ms, rs, sd)


def _round_model(m: ir.Model, fields: Dict[str, str]) -> None:
    local = dict(fields)
    for d in m.local_transformations:
        local[d.name] = getattr(d, "optype", None) or "continuous"
    if isinstance(m, ir.TreeModel):
        regression = m.function_name != "classification"
        ft = getattr(m, "flat", None)
        if ft is not None and ft._root is None:
            _round_flat(ft, local, regression)
            return
        stack = [m.root]
        while stack:
            n = stack.pop()
            _round_predicate(n.predicate, local)
            if regression:
                n.score = _round_value(n.score)
            stack.extend(n.children)
    elif isinstance(m, ir.RegressionModel):
        for t in m.tables:
            t.intercept = float(np.float32(t.intercept))
            for p in t.numeric:
                p.coefficient = float(np.float32(p.coefficient))
            for p in t.categorical:
                p.coefficient = float(np.float32(p.coefficient))
            for p in t.terms:
                p.coefficient = float(np.float32(p.coefficient))
    elif isinstance(m, ir.MiningModel):
        for s in m.segments:
            s.weight = float(np.float32(s.weight))
            _round_predicate(s.predicate, local)


def _walk(models: Iterable[ir.Model], inherited: Optional[str], fields: Dict[str, str]) -> None:
    for m in models:
        ctx = m.math_context or inherited
        if ctx == "float":
            m.math_context = "float"
            _round_model(m, fields)
        if isinstance(m, ir.MiningModel):
            _walk([s.model for s in m.segments], ctx, fields)


def apply_math_context(doc: ir.PMMLDocument) -> ir.PMMLDocument:
    """Round the float-context models of ``doc`` in place (module docstring); returns ``doc``."""
    if not any(_has_context(m) for m in doc.models):
        return doc
    fields = {n: f.optype for n, f in doc.data_fields.items()}
    for d in doc.transformations:
        fields[d.name] = getattr(d, "optype", None) or "continuous"
    _walk(doc.models, None, fields)
    return doc


def _has_context(m: ir.Model) -> bool:
    if m.math_context is not None:
        return True
    return isinstance(m, ir.MiningModel) and any(_has_context(s.model) for s in m.segments)


def is_float(m: ir.Model) -> bool:
    return getattr(m, "math_context", None) == "float"


__all__ = ["apply_math_context", "is_float"]
