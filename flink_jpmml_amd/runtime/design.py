"""Regression-family models on the device through a *design matrix*.

``RegressionModel`` tables with categorical predictors, interaction terms (``PredictorTerm``) or
non-unit exponents, and ``GeneralRegressionModel`` (PPMatrix / ParamMatrix GLMs) are all linear in
a set of per-row *design columns*:

* ``x^e`` for a numeric predictor / covariate (``Apply("pow")``; ``e == 1`` reads ``x`` itself),
* ``[x == v]`` for a categorical predictor / factor level (``NormDiscrete`` with
  ``mapMissingTo=0``: a missing categorical contributes 0, the PMML rule the oracle follows),
* products of those for interaction terms and multi-predictor GLM parameters.

JPMML evaluates these tables per record inside ``ModelEvaluator.evaluate``
(`S/api/PmmlModel.scala:159-160`). Here the design columns become a derive program
(``ops/csrc/derive.hip``, :mod:`.derive`) and the model a *dense* ``RegressionModel`` over them,
scored by the fused GEMV + link kernel (``ops/csrc/linear.hip``). A missing numeric predictor turns
its design column into NaN and the linear kernel invalidates the row — the oracle's
"missing numeric predictor ⇒ no prediction" rule.

GLM links map onto the RegressionModel normalisations (identity → none, log → exp, logit, probit,
cloglog, power 0/1); ``multinomialLogistic`` is a softmax over per-category tables with a zero
table for the reference category.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

from ..models.regression import GeneralRegressionEvaluator, RegressionEvaluator
from ..pmml import ir
from .plans import NotLowerable

_GLM_LINKS = {None: "none", "identity": "none", "log": "exp", "logit": "logit", "probit": "probit",
              "cloglog": "cloglog", "loglog": "loglog"}
# binomial GLM with the reference category FIRST: P(ref) = 1 - F(η) = F'(-η)
_MIRRORED = {"logit": "logit", "probit": "probit", "cloglog": "loglog", "loglog": "cloglog"}


class _Design:
    def __init__(self):
        self.defs: Dict[str, ir.DerivedField] = {}
        self.keys: Dict[tuple, str] = {}

    def column(self, key: tuple, expr: ir.Expression) -> str:
        name = self.keys.get(key)
        if name is None:
            name = f"__design{len(self.keys)}"
            self.keys[key] = name
            self.defs[name] = ir.DerivedField(name, "continuous", "double", expr)
        return name

    def power(self, field: str, e: float) -> Tuple[tuple, ir.Expression]:
        if e == 1.0:
            return ("x", field), ir.FieldRef(field)
        return ("pow", field, e), ir.Apply("pow", [ir.FieldRef(field), ir.Constant(repr(float(e)))])

    @staticmethod
    def level(field: str, value) -> Tuple[tuple, ir.Expression]:
        return ("lvl", field, str(value)), ir.NormDiscrete(field, str(value), map_missing_to=0.0)

    def product(self, parts: List[Tuple[tuple, ir.Expression]]) -> Tuple[tuple, Optional[ir.Expression]]:
        """Design column of a product (None expression: the empty product, an intercept)."""
        if not parts:
            return ("one",), None
        parts = sorted(parts, key=lambda p: repr(p[0]))
        expr = parts[0][1]
        for _, e in parts[1:]:
            expr = ir.Apply("*", [expr, e])
        return tuple(p[0] for p in parts), expr

    def name_of(self, key: tuple, expr: ir.Expression) -> str:
        if isinstance(expr, ir.FieldRef) and expr.map_missing_to is None:
            return expr.field  # a plain input (or derived) field: no new column
        return self.column(key, expr)


def _regression_tables(ev: RegressionEvaluator, d: _Design) -> List[ir.RegressionTable]:
    out = []
    for t in ev.rm.tables:
        coef: Dict[str, float] = {}

        def add(name: str, c: float) -> None:
            coef[name] = coef.get(name, 0.0) + c

        for p in t.numeric:
            add(d.name_of(*d.power(p.name, p.exponent)), p.coefficient)
        for p in t.categorical:
            add(d.name_of(*d.level(p.name, p.value)), p.coefficient)
        for term in t.terms:
            if not term.fields:
                raise NotLowerable("empty PredictorTerm")
            add(d.name_of(*d.product([d.power(f, 1.0) for f in term.fields])), term.coefficient)
        out.append(ir.RegressionTable(t.intercept, t.target_category,
                                      [ir.NumericPredictor(n, c) for n, c in coef.items()]))
    return out


def _glm_tables(ev: GeneralRegressionEvaluator, d: _Design) -> Tuple[List[ir.RegressionTable], str]:
    gm = ev.gm
    param_col: Dict[str, Optional[str]] = {}
    for param in dict.fromkeys([p for p, _, _ in gm.p_cells]):
        parts = []
        for pred, val in ev.pp.get(param, []):
            if pred in gm.factors:
                parts.append(d.level(pred, val))
            else:
                parts.append(d.power(pred, float(val) if val is not None else 1.0))
        key, expr = d.product(parts)
        param_col[param] = None if expr is None else d.name_of(key, expr)

    def table(category) -> ir.RegressionTable:
        icpt = gm.offset_value
        coef: Dict[str, float] = {}
        for param, tc, beta in gm.p_cells:
            if tc != category:
                continue
            col = param_col[param]
            if col is None:
                icpt += beta
            else:
                coef[col] = coef.get(col, 0.0) + beta
        return ir.RegressionTable(icpt, category, [ir.NumericPredictor(n, c) for n, c in coef.items()])

    if ev.kind != "classification":
        lf = gm.link_function
        if gm.model_type in ("regression", "generalLinear"):
            norm = "none"
        elif lf == "power":
            p = gm.link_power if gm.link_power is not None else 1.0
            if p not in (0.0, 1.0):
                raise NotLowerable(f"power link with power {p} is host-only")
            norm = "exp" if p == 0.0 else "none"
        elif lf in _GLM_LINKS:
            norm = _GLM_LINKS[lf]
        else:
            raise NotLowerable(f"GLM linkFunction {lf!r} is host-only")
        return [table(None)], norm
    if gm.model_type == "ordinalMultinomial":
        # one table per category: cut point + shared slopes (cells without a targetCategory); the
        # last category's table is a placeholder — the cumulative epilogue gives it 1 - F(η_{J-2})
        shared = table(None)
        tabs = []
        for c in ev.categories[:-1]:
            own = table(c)
            coef: Dict[str, float] = {}
            for p in own.numeric + shared.numeric:
                coef[p.name] = coef.get(p.name, 0.0) + p.coefficient
            tabs.append(ir.RegressionTable(own.intercept + shared.intercept - gm.offset_value, c,
                                           [ir.NumericPredictor(n, w) for n, w in coef.items()]))
        tabs.append(ir.RegressionTable(0.0, ev.categories[-1], []))
        return tabs, f"cumulative:{gm.cumulative_link or 'logit'}"
    if gm.model_type == "generalizedLinear":
        # binomial: the PMML two-table rule p0 = F(y0), p1 = 1 - p0 (LinearPlan's EPI_LOGISTIC2)
        # with the tables in category order; a reference category listed first gets y0 = -η
        # through the mirrored link (identity: y0 = 1 - η)
        ref, event = ev.binomial_roles()
        lf = gm.link_function or "logit"
        if lf not in _MIRRORED and lf != "identity":
            raise NotLowerable(f"classification generalizedLinear linkFunction {lf!r} is host-only")
        own, shared = table(event), table(None)
        coef: Dict[str, float] = {}
        for p in own.numeric + shared.numeric:
            coef[p.name] = coef.get(p.name, 0.0) + p.coefficient
        icpt = own.intercept + (shared.intercept - gm.offset_value if any(tc is None for _, tc, _ in gm.p_cells)
                                else 0.0)
        if ev.categories[0] == event:
            first = ir.RegressionTable(icpt, event, [ir.NumericPredictor(n, w) for n, w in coef.items()])
            norm = _GLM_LINKS[lf]
        elif lf == "identity":
            first = ir.RegressionTable(1.0 - icpt, ref, [ir.NumericPredictor(n, -w) for n, w in coef.items()])
            norm = "none"
        else:
            first = ir.RegressionTable(-icpt, ref, [ir.NumericPredictor(n, -w) for n, w in coef.items()])
            norm = _MIRRORED[lf]
        second = ir.RegressionTable(0.0, ev.categories[1], [])
        return [first, second], norm
    if gm.model_type != "multinomialLogistic":
        raise NotLowerable(f"classification GeneralRegressionModel {gm.model_type!r} is host-only")
    tabs = []
    for c in ev.categories:
        tabs.append(ir.RegressionTable(0.0, c, []) if c == gm.target_reference_category else table(c))
    return tabs, "softmax"


def _naive_bayes_tables(ev, d: _Design) -> Tuple[List[ir.RegressionTable], str]:
    """log n_j + Σ_i log P(x_i | T_j), each factor linear in design columns; softmax."""
    import math

    import numpy as np

    if (ev.counts <= 0).any():
        raise NotLowerable("NaiveBayes class with a zero count")
    K = len(ev.categories)
    coef: List[Dict[str, float]] = [dict() for _ in range(K)]

    def add(name: str, w) -> None:
        for j in range(K):
            coef[j][name] = coef[j].get(name, 0.0) + float(w[j])

    for inp in ev.nb.inputs:
        f = inp.field
        if inp.gaussian:
            g = ev.gaussian_params(inp)
            if np.isnan(g).any() or (g[:, 1] <= 0).any():
                raise NotLowerable(f"NaiveBayes input {f!r}: Gaussian stats missing for a class")
            mu, var = g[:, 0], g[:, 1]
            add(d.column(("present", f), ir.Apply("isNotMissing", [ir.FieldRef(f)])),
                -0.5 * np.log(2 * math.pi * var) - mu * mu / (2 * var))
            add(d.column(("x0", f), ir.FieldRef(f, map_missing_to="0")), mu / var)
            add(d.column(("x2", f), ir.Apply("pow", [ir.FieldRef(f), ir.Constant("2")], map_missing_to="0")),
                -1.0 / (2 * var))
        else:
            for v, lp in ev.level_log_probs(inp):
                if not np.isfinite(lp).all():
                    raise NotLowerable("NaiveBayes zero probability without a threshold")
                add(d.name_of(*d.level(f, v)), lp)
    tabs = [ir.RegressionTable(float(np.log(ev.counts[j])), c, [ir.NumericPredictor(n, w) for n, w in coef[j].items()])
            for j, c in enumerate(ev.categories)]
    return tabs, "softmax"


def needs_design(ev) -> bool:
    from ..models.naive_bayes import NaiveBayesEvaluator

    if isinstance(ev, (GeneralRegressionEvaluator, NaiveBayesEvaluator)):
        return True
    return isinstance(ev, RegressionEvaluator) and not ev.is_dense_linear()


def design_layout(compiled):
    """-> (:class:`~.derive.FieldLayout` of the design columns, dense ``RegressionEvaluator`` over
    them). The layout always carries a derive program unless every column is a plain field."""
    from .derive import FieldLayout, build_program_layout, collect_derived

    from ..models.naive_bayes import NaiveBayesEvaluator

    ev = compiled.evaluator
    d = _Design()
    if isinstance(ev, NaiveBayesEvaluator):
        tables, norm = _naive_bayes_tables(ev, d)
        base = {f.name: getattr(ev.nb, f.name) for f in dataclasses.fields(ir.Model)}
        base["element"] = "RegressionModel"
        model = ir.RegressionModel(**base, normalization_method=norm, tables=tables)
    elif isinstance(ev, GeneralRegressionEvaluator):
        tables, norm = _glm_tables(ev, d)
        gm = ev.gm
        base = {f.name: getattr(gm, f.name) for f in dataclasses.fields(ir.Model)}
        base["element"] = "RegressionModel"
        model = ir.RegressionModel(**base, normalization_method=norm, tables=tables)
    elif isinstance(ev, RegressionEvaluator):
        model = dataclasses.replace(ev.rm, tables=_regression_tables(ev, d))
    else:
        raise NotLowerable(f"no design lowering for {type(ev).__name__}")
    dense = RegressionEvaluator(model, compiled.schema)
    if not dense.numeric_fields:
        raise NotLowerable("regression without predictors")
    defs = collect_derived(compiled)
    clash = set(defs) & set(d.defs)
    if clash:
        raise NotLowerable(f"derived field names clash with design columns: {sorted(clash)}")
    defs.update(d.defs)
    layout: FieldLayout = build_program_layout(compiled, defs, list(dense.numeric_fields))
    layout.evaluator = dense
    return layout, dense
