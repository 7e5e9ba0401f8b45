"""SupportVectorMachineModel — oracle and kernel-matrix lowering.

Per machine: ``f(x) = Σ_i α_i · K(x, sv_i) + b`` (``SupportVectors`` representation) or
``f(x) = Σ_j c_j · x_j + b`` (``Coefficients``, linear kernel), with kernels ``linear`` x·y,
``polynomial`` (γ·x·y + c₀)^d, ``radialBasis`` exp(−γ‖x−y‖²), ``sigmoid`` tanh(γ·x·y + c₀).

Classification: binary / ``OneAgainstAll`` machines predict ``targetCategory`` when
f(x) < threshold, else ``alternateTargetCategory`` (PMML 4.x); ``OneAgainstOne`` counts votes
across machines (ties → first category in declaration order). With ``maxWins`` the comparison is
reversed. Regression returns f(x) of the single machine.
"""

from __future__ import annotations

from typing import List

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from .base import ModelEvaluator, ModelResult


def kernel_matrix(kind: str, X: np.ndarray, S: np.ndarray, gamma: float, coef0: float, degree: float) -> np.ndarray:
    if kind == "radialBasis":
        d2 = (X * X).sum(1)[:, None] - 2.0 * X @ S.T + (S * S).sum(1)[None, :]
        return np.exp(-gamma * np.maximum(d2, 0.0))
    G = X @ S.T
    if kind == "linear":
        return G
    if kind == "polynomial":
        return np.power(gamma * G + coef0, degree)
    if kind == "sigmoid":
        return np.tanh(gamma * G + coef0)
    raise UnsupportedFeatureException(f"SVM kernel {kind!r}")


class SvmEvaluator(ModelEvaluator):
    def __init__(self, model: ir.SupportVectorMachineModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.sm = model
        self.fields: List[str] = model.vector_fields or list(self.active_fields)
        self.sv_ids: List[str] = list(model.vectors.keys())
        self.S = np.array([model.vectors[i] for i in self.sv_ids], dtype=np.float64) if self.sv_ids else \
            np.zeros((0, len(self.fields)))
        # dual-coefficient matrix A[sv, machine] + intercepts b[machine]
        M = len(model.machines)
        self.A = np.zeros((len(self.sv_ids), M))
        self.b = np.zeros(M)
        self.linear_coef = np.zeros((len(self.fields), M))
        pos = {sid: i for i, sid in enumerate(self.sv_ids)}
        for m, mach in enumerate(model.machines):
            self.b[m] = mach.intercept
            if model.representation == "Coefficients":
                if len(mach.coefficients) != len(self.fields):
                    raise UnsupportedFeatureException("Coefficients representation needs one coefficient per field")
                self.linear_coef[:, m] = mach.coefficients
            else:
                for sid, c in zip(mach.vector_ids, mach.coefficients):
                    self.A[pos[sid], m] += c
        if self.kind == "classification":
            cats = self.classification_categories()
            for mach in model.machines:
                for c in (mach.target_category, mach.alternate_target_category):
                    if c is not None and c not in cats:
                        cats.append(c)
            self.categories = cats
        else:
            self.categories = None

    def decision_values(self, X: np.ndarray) -> np.ndarray:
        k = self.sm.kernel
        if self.sm.representation == "Coefficients":
            return X @ self.linear_coef + self.b[None, :]
        K = kernel_matrix(k.kind, X, self.S, k.gamma, k.coef0, k.degree)
        return K @ self.A + self.b[None, :]

    def _evaluate(self, cols: Columns) -> ModelResult:
        X = np.stack([cols.get(f) for f in self.fields], axis=1)
        miss = np.any(np.isnan(X), axis=1)
        D = self.decision_values(np.nan_to_num(X))
        return self.finish(D, ~miss)

    def finish(self, D: np.ndarray, valid: np.ndarray) -> ModelResult:
        n = D.shape[0]
        if self.kind != "classification":
            y = D[:, 0]
            return ModelResult("regression", np.where(valid, y, NAN), valid.copy())
        cats = self.categories
        machines = self.sm.machines
        votes = np.zeros((n, len(cats)))
        for m, mach in enumerate(machines):
            thr = mach.threshold if mach.threshold is not None else self.sm.threshold
            first = D[:, m] < thr
            if self.sm.max_wins:
                first = ~first
            t = cats.index(mach.target_category)
            if mach.alternate_target_category is not None:
                a = cats.index(mach.alternate_target_category)
                votes[first, t] += 1
                votes[~first, a] += 1
            else:
                # OneAgainstAll without alternate: the machine votes for its category when it fires
                votes[first, t] += 1
        lab = np.argmax(votes, axis=1).astype(np.float64)
        return ModelResult("classification", np.where(valid, lab, NAN), valid.copy(), categories=cats,
                           probs=None, extra={"votes": votes})
