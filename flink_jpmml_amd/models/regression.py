"""RegressionModel (linear / logistic) and GeneralRegressionModel (GLM subset).

``y_k = intercept_k + Σ coef·x^exp + Σ coef·[x == category] + Σ coef·Πfields`` per
``RegressionTable``; then ``normalizationMethod``:

* regression: ``none``, ``logit`` 1/(1+e^-y), ``exp``, ``probit`` Φ(y), ``cloglog`` 1−exp(−e^y),
  ``loglog`` exp(−e^−y), ``cauchit`` ½+atan(y)/π;
* classification: ``softmax`` / ``simplemax`` across tables; for the element-wise links with two
  tables the first category gets f(y₀) and the second 1 − f(y₀); with more tables each gets f(y_k)
  (``none``: raw y_k).

A missing numeric predictor makes the prediction missing (PMML spec); a missing categorical
predictor contributes 0.
"""

from __future__ import annotations

import math
from typing import List

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from ..pmml.mathcontext import is_float
from .base import ModelEvaluator, ModelResult

_SQRT2 = math.sqrt(2.0)


def _erf(x: np.ndarray) -> np.ndarray:
    from scipy.special import erf  # scipy is available in the image

    return erf(x)


def link(method: str, y: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore", invalid="ignore"):
        if method in ("none", None):
            return y
        if method == "logit":
            return 1.0 / (1.0 + np.exp(-y))
        if method == "exp":
            return np.exp(y)
        if method == "probit":
            return 0.5 * (1.0 + _erf(y / _SQRT2))
        if method == "cloglog":
            return 1.0 - np.exp(-np.exp(y))
        if method == "loglog":
            return np.exp(-np.exp(-y))
        if method == "cauchit":
            return 0.5 + np.arctan(y) / math.pi
    raise UnsupportedFeatureException(f"normalizationMethod {method!r}")


class RegressionEvaluator(ModelEvaluator):
    def __init__(self, model: ir.RegressionModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.rm = model
        if not model.tables:
            raise UnsupportedFeatureException("RegressionModel without RegressionTable")
        if self.kind == "classification":
            cats = [t.target_category for t in model.tables]
            self.categories = [str(c) for c in cats]
        else:
            self.categories = None
        # dense lowering: y = X @ W + b for pure numeric (exponent 1) tables; used by the GPU plan
        self.numeric_fields: List[str] = []
        for t in model.tables:
            for p in t.numeric:
                if p.name not in self.numeric_fields:
                    self.numeric_fields.append(p.name)

    def is_dense_linear(self) -> bool:
        return all(not t.categorical and not t.terms and all(p.exponent == 1.0 for p in t.numeric)
                   for t in self.rm.tables)

    def dense_weights(self) -> tuple:
        F, T = len(self.numeric_fields), len(self.rm.tables)
        W = np.zeros((F, T))
        b = np.zeros(T)
        for k, t in enumerate(self.rm.tables):
            b[k] = t.intercept
            for p in t.numeric:
                W[self.numeric_fields.index(p.name), k] += p.coefficient
        return W, b

    def raw_scores(self, cols: Columns) -> tuple:
        if is_float(self.rm):
            return self._raw_scores_f32(cols)
        n = cols.n
        Y = np.zeros((n, len(self.rm.tables)))
        miss = np.zeros(n, dtype=bool)
        for k, t in enumerate(self.rm.tables):
            y = np.full(n, t.intercept)
            for p in t.numeric:
                x = cols.get(p.name)
                miss |= np.isnan(x)
                y = y + p.coefficient * (x if p.exponent == 1.0 else np.power(x, p.exponent))
            for p in t.categorical:
                x = cols.get(p.name)
                lit = self.schema.lookup(p.name, p.value)
                y = y + np.where(x == lit, p.coefficient, 0.0)
            for term in t.terms:
                prod = np.ones(n)
                for f in term.fields:
                    x = cols.get(f)
                    miss |= np.isnan(x)
                    prod = prod * x
                y = y + term.coefficient * prod
            Y[:, k] = y
        return Y, miss

    def _raw_scores_f32(self, cols: Columns) -> tuple:
        """``x-mathContext="float"``: every product and partial sum in float32, in term order."""
        n = cols.n
        f32 = np.float32
        Y = np.zeros((n, len(self.rm.tables)), dtype=np.float32)
        miss = np.zeros(n, dtype=bool)
        for k, t in enumerate(self.rm.tables):
            y = np.full(n, f32(t.intercept), dtype=np.float32)
            for p in t.numeric:
                x = cols.get(p.name).astype(np.float32)
                miss |= np.isnan(x)
                xe = x if p.exponent == 1.0 else np.power(x, f32(p.exponent))
                y = y + f32(p.coefficient) * xe
            for p in t.categorical:
                x = cols.get(p.name)
                lit = self.schema.lookup(p.name, p.value)
                y = y + np.where(x == lit, f32(p.coefficient), f32(0.0))
            for term in t.terms:
                prod = np.ones(n, dtype=np.float32)
                for f in term.fields:
                    x = cols.get(f).astype(np.float32)
                    miss |= np.isnan(x)
                    prod = prod * x
                y = y + f32(term.coefficient) * prod
            Y[:, k] = y
        return Y, miss

    def _evaluate(self, cols: Columns) -> ModelResult:
        Y, miss = self.raw_scores(cols)
        return self.finish(Y, ~miss)

    def finish(self, Y: np.ndarray, valid: np.ndarray) -> ModelResult:
        norm = self.rm.normalization_method
        if self.kind != "classification":
            y = link(norm, Y[:, 0])
            return ModelResult("regression", np.where(valid, y, NAN), valid & np.isfinite(y))
        T = Y.shape[1]
        with np.errstate(over="ignore", invalid="ignore"):
            if norm == "softmax":
                Z = Y - Y.max(axis=1, keepdims=True)
                E = np.exp(Z)
                P = E / E.sum(axis=1, keepdims=True)
            elif norm == "simplemax":
                P = Y / Y.sum(axis=1, keepdims=True)
            elif norm.startswith("cumulative:"):  # ordinal GLM lowered to tables (runtime/design.py)
                cum = link(norm.split(":", 1)[1], Y)
                cum[:, -1] = 1.0
                P = np.diff(cum, axis=1, prepend=0.0)
            elif T == 2 and norm != "none":
                p0 = link(norm, Y[:, 0])
                P = np.stack([p0, 1.0 - p0], axis=1)
            elif T == 2 and norm == "none":
                P = np.stack([Y[:, 0], 1.0 - Y[:, 0]], axis=1)
            else:
                P = link(norm, Y)
        lab = np.argmax(np.nan_to_num(P, nan=-np.inf), axis=1).astype(np.float64)
        ok = valid & np.all(np.isfinite(P), axis=1)
        return ModelResult("classification", np.where(ok, lab, NAN), ok, categories=self.categories,
                           probs=np.where(ok[:, None], P, NAN))


class GeneralRegressionEvaluator(ModelEvaluator):
    """GeneralRegressionModel for ``regression``, ``generalLinear``, ``generalizedLinear``
    (identity/log/logit/probit/cloglog/loglog/power links; as a binomial classifier too),
    ``multinomialLogistic`` and
    ``ordinalMultinomial`` (cumulative logit/probit/cloglog/loglog/cauchit). Parity unpinned (no
    JPMML here): follows the PMML 4.4 GeneralRegression text."""

    def __init__(self, model: ir.GeneralRegressionModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.gm = model
        if model.model_type not in ("regression", "generalLinear", "generalizedLinear", "multinomialLogistic",
                                    "ordinalMultinomial"):
            raise UnsupportedFeatureException(f"GeneralRegressionModel modelType {model.model_type!r}")
        # parameter -> list of (predictor, value)
        self.pp: dict = {}
        for pred, param, val in model.pp_cells:
            self.pp.setdefault(param, []).append((pred, val))
        self.cats: List[str] = []
        for _, tc, _ in model.p_cells:
            if tc is not None and tc not in self.cats:
                self.cats.append(tc)
        if self.kind == "classification":
            all_cats = self.classification_categories() or list(self.cats)
            if model.target_reference_category and model.target_reference_category not in all_cats:
                all_cats.append(model.target_reference_category)
            self.categories = all_cats
        else:
            self.categories = None

    def _design(self, cols: Columns, param: str) -> tuple:
        n = cols.n
        col = np.ones(n)
        miss = np.zeros(n, dtype=bool)
        for pred, val in self.pp.get(param, []):
            x = cols.get(pred)
            if pred in self.gm.factors:
                col = col * (x == self.schema.lookup(pred, val)).astype(np.float64)
            else:
                miss |= np.isnan(x)
                e = float(val) if val is not None else 1.0
                col = col * np.power(x, e)
        return col, miss

    def _linear(self, cols: Columns, category) -> tuple:
        n = cols.n
        eta = np.full(n, self.gm.offset_value)
        miss = np.zeros(n, dtype=bool)
        for param, tc, beta in self.gm.p_cells:
            if tc != category:
                continue
            col, m = self._design(cols, param)
            eta = eta + beta * col
            miss |= m
        return eta, miss

    def _evaluate(self, cols: Columns) -> ModelResult:
        gm = self.gm
        if self.kind != "classification":
            eta, miss = self._linear(cols, None)
            lf = gm.link_function
            if gm.model_type in ("regression", "generalLinear") or lf in (None, "identity"):
                y = eta
            elif lf == "log":
                y = np.exp(eta)
            elif lf == "logit":
                y = 1.0 / (1.0 + np.exp(-eta))
            elif lf == "probit":
                y = link("probit", eta)
            elif lf in ("cloglog", "loglog"):
                y = link(lf, eta)
            elif lf == "power":
                p = gm.link_power if gm.link_power is not None else 1.0
                y = np.exp(eta) if p == 0 else np.power(eta, 1.0 / p)
            else:
                raise UnsupportedFeatureException(f"linkFunction {lf!r}")
            return ModelResult("regression", np.where(miss, NAN, y), ~miss & np.isfinite(y))
        cats = self.categories
        n = cols.n
        if gm.model_type == "ordinalMultinomial":
            return self._ordinal(cols)
        if gm.model_type == "generalizedLinear":
            return self._binomial(cols)
        etas = np.zeros((n, len(cats)))
        miss = np.zeros(n, dtype=bool)
        for k, c in enumerate(cats):
            if c == gm.target_reference_category:
                continue
            e, m = self._linear(cols, c)
            etas[:, k] = e
            miss |= m
        if gm.model_type == "multinomialLogistic":
            Z = etas - etas.max(axis=1, keepdims=True)
            E = np.exp(Z)
            P = E / E.sum(axis=1, keepdims=True)
        else:
            raise UnsupportedFeatureException(f"classification GeneralRegressionModel {gm.model_type!r}")
        lab = np.argmax(P, axis=1).astype(np.float64)
        ok = ~miss
        return ModelResult("classification", np.where(ok, lab, NAN), ok, categories=cats,
                           probs=np.where(ok[:, None], P, NAN))

    def binomial_roles(self) -> tuple:
        """``(reference, event)`` categories of a classification ``generalizedLinear`` model: exactly
        two categories; the reference is ``targetReferenceCategory`` (default: the last one)."""
        cats = self.categories
        if len(cats) != 2:
            raise UnsupportedFeatureException(f"classification generalizedLinear needs 2 categories, got {len(cats)}")
        ref = self.gm.target_reference_category if self.gm.target_reference_category is not None else cats[-1]
        if ref not in cats:
            raise UnsupportedFeatureException(f"targetReferenceCategory {ref!r} is not a target category")
        return ref, cats[1] if cats[0] == ref else cats[0]

    def _binomial(self, cols: Columns) -> ModelResult:
        """Classification ``generalizedLinear`` (binomial GLM): ``P(event) = F(η)`` with F the
        inverse ``linkFunction`` and η over the event category's PCells plus the cells without a
        targetCategory (exports use one or the other); the reference category takes ``1 − P``."""
        gm = self.gm
        cats = self.categories
        ref, event = self.binomial_roles()
        lf = gm.link_function or "logit"
        names = {"logit": "logit", "probit": "probit", "cloglog": "cloglog", "loglog": "loglog", "identity": "none"}
        if lf not in names:
            raise UnsupportedFeatureException(f"classification generalizedLinear linkFunction {lf!r}")
        eta, miss = self._linear(cols, event)
        if any(tc is None for _, tc, _ in gm.p_cells):
            e0, m0 = self._linear(cols, None)
            eta, miss = eta + e0 - gm.offset_value, miss | m0  # offset counted once
        p = link(names[lf], eta)
        P = np.empty((cols.n, 2))
        P[:, cats.index(event)] = p
        P[:, cats.index(ref)] = 1.0 - p
        lab = np.argmax(np.nan_to_num(P, nan=-np.inf), axis=1).astype(np.float64)
        ok = ~miss & np.isfinite(P).all(axis=1)
        return ModelResult("classification", np.where(ok, lab, NAN), ok, categories=cats,
                           probs=np.where(ok[:, None], P, NAN))

    def _ordinal(self, cols: Columns) -> ModelResult:
        """``ordinalMultinomial``: cumulative link over the ordered categories. Category j < J-1 has
        ``η_j = offset + Σ β`` over its own cells (the cut point) and the cells without a
        targetCategory (the shared slopes); ``P(Y ≤ j) = F(η_j)`` with F the inverse
        ``cumulativeLink``; ``P(j) = P(Y ≤ j) − P(Y ≤ j−1)``, the last category takes the rest."""
        gm = self.gm
        cats = self.categories
        n, J = cols.n, len(cats)
        F = gm.cumulative_link or "logit"
        if F not in ("logit", "probit", "cloglog", "loglog", "cauchit"):
            raise UnsupportedFeatureException(f"cumulativeLink {F!r}")
        shared, miss = self._linear(cols, None)
        cum = np.ones((n, J))
        for j, c in enumerate(cats[:-1]):
            e, m = self._linear(cols, c)
            miss |= m
            cum[:, j] = link(F, e + shared - gm.offset_value)  # offset counted once
        P = np.diff(cum, axis=1, prepend=0.0)
        lab = np.argmax(np.nan_to_num(P, nan=-np.inf), axis=1).astype(np.float64)
        ok = ~miss & np.isfinite(P).all(axis=1)
        return ModelResult("classification", np.where(ok, lab, NAN), ok, categories=cats,
                           probs=np.where(ok[:, None], P, NAN))
