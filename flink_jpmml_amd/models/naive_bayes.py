"""NaiveBayesModel (PMML 4.4): ``P(T_j | x) ∝ n_j · Π_i P(x_i | T_j)``.

* categorical input ``x_i = v``: ``P = count(v, T_j) / n_j`` (``PairCounts``; ``n_j`` from
  ``BayesOutput``), a zero probability replaced by the model ``threshold``; a value without
  ``PairCounts`` contributes nothing;
* continuous input: ``GaussianDistribution`` density (zero → ``threshold``);
* a missing input contributes nothing (its factor is skipped).

Evaluated in log space and softmax-normalised. JPMML evaluates it per record
(`S/api/PmmlModel.scala:159-160`); here it is a host oracle plus a device lowering: every factor is
linear in per-row design columns (level indicators; ``1[present]``, ``x``, ``x²`` of the Gaussian
log-density), so ``runtime/design.py`` turns the model into a derive program + dense GEMV with a
softmax epilogue. Parity unpinned (no JPMML here): follows the specification text.
"""

from __future__ import annotations

import math
from typing import List

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from .base import ModelEvaluator, ModelResult


class NaiveBayesEvaluator(ModelEvaluator):
    def __init__(self, model: ir.NaiveBayesModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.nb = model
        if self.kind != "classification":
            raise UnsupportedFeatureException("NaiveBayesModel must be a classification model")
        cats: List[str] = [c for c in self.classification_categories() if c in model.target_counts]
        cats += [c for c in model.target_counts if c not in cats]
        self.categories = cats
        self.counts = np.array([model.target_counts[c] for c in cats], dtype=np.float64)
        self.log_threshold = math.log(model.threshold) if model.threshold > 0 else -math.inf

    def level_log_probs(self, inp: ir.BayesInput) -> List[tuple]:
        """``[(value, log P(value | T_j) per class)]`` for a categorical input."""
        out = []
        for v, tc in inp.pair_counts.items():
            with np.errstate(divide="ignore"):
                p = np.array([tc.get(c, 0.0) for c in self.categories]) / self.counts
                lp = np.where(p > 0, np.log(np.where(p > 0, p, 1.0)), self.log_threshold)
            out.append((v, lp))
        return out

    def gaussian_params(self, inp: ir.BayesInput) -> np.ndarray:
        """``[classes, 2]`` (mean, variance); classes without a stat get NaN."""
        return np.array([inp.gaussian.get(c, (NAN, NAN)) for c in self.categories], dtype=np.float64)

    def _evaluate(self, cols: Columns) -> ModelResult:
        n = cols.n
        with np.errstate(divide="ignore"):
            L = np.tile(np.log(self.counts), (n, 1))
        for inp in self.nb.inputs:
            x = cols.get(inp.field)
            present = ~np.isnan(x)
            if inp.gaussian:
                g = self.gaussian_params(inp)
                mu, var = g[:, 0][None, :], g[:, 1][None, :]
                with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
                    lp = -0.5 * np.log(2 * math.pi * var) - (x[:, None] - mu) ** 2 / (2 * var)
                lp = np.where(np.isneginf(lp), self.log_threshold, lp)
                L += np.where(present[:, None], np.nan_to_num(lp, nan=0.0), 0.0)
            else:
                for v, lp in self.level_log_probs(inp):
                    hit = present & (x == self.schema.lookup(inp.field, v))
                    L += np.where(hit[:, None], lp[None, :], 0.0)
        with np.errstate(invalid="ignore"):
            Z = L - L.max(axis=1, keepdims=True)
            E = np.exp(Z)
            P = E / E.sum(axis=1, keepdims=True)
        ok = np.isfinite(P).all(axis=1)
        lab = np.argmax(np.nan_to_num(P, nan=-1.0), axis=1).astype(np.float64)
        return ModelResult("classification", np.where(ok, lab, NAN), ok, categories=self.categories,
                           probs=np.where(ok[:, None], P, NAN))
