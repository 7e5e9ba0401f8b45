"""ClusteringModel (center-based), the model family the reference exercises end to end
(`A/kmeans.xml:43-73`, goldens `T/api/PmmlModelSpec.scala:50-83`).

Semantics (PMML 4.x ClusteringModel):

* per-field comparison ``c(x, y)``: ``absDiff`` |x−y|, ``gaussSim`` exp(−ln2·z²/s²), ``delta``
  (0 if equal else 1), ``equal`` (1 if equal else 0);
* metric: ``squaredEuclidean`` Σw·c², ``euclidean`` √Σw·c², ``cityBlock`` Σw·c,
  ``chebychev`` max w·c, ``minkowski`` (Σw·c^p)^(1/p);
* missing inputs are skipped and the sum is rescaled by ``Σq / Σq_present`` where ``q`` are the
  ``MissingValueWeights`` (default 1) — SURVEY §2.8 K1;
* winner = argmin distance (``kind="distance"``) / argmax similarity; the entity id is the
  cluster ``id`` attribute or its 1-based position.
"""

from __future__ import annotations

from typing import List

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from .base import ModelEvaluator, ModelResult

_DISTANCE_METRICS = ("euclidean", "squaredEuclidean", "cityBlock", "chebychev", "minkowski")
_SIMILARITY_METRICS = ("simpleMatching", "jaccard", "tanimoto", "binarySimilarity")


class ClusteringEvaluator(ModelEvaluator):
    kind = "clustering"

    def __init__(self, model: ir.ClusteringModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.kind = "clustering"
        m = model
        fields = [f for f in m.fields if f.is_center_field] or [
            ir.ClusteringField(f) for f in self.active_fields
        ]
        self.fields: List[str] = [f.field for f in fields]
        self.weights = np.array([f.weight for f in fields], dtype=np.float64)
        self.compare = [f.compare_function or m.compare_function for f in fields]
        self.scales = np.array([f.similarity_scale if f.similarity_scale is not None else 1.0 for f in fields])
        self.centers = np.array([c.center for c in m.clusters], dtype=np.float64)
        if self.centers.ndim != 2 or self.centers.shape[1] != len(fields):
            raise UnsupportedFeatureException(
                f"cluster centers have shape {self.centers.shape}, expected [K, {len(fields)}]")
        self.entity_ids = [c.id if c.id is not None else str(i + 1) for i, c in enumerate(m.clusters)]
        self.cluster_names = [c.name for c in m.clusters]
        q = m.missing_value_weights
        self.missing_weights = np.array(q, dtype=np.float64) if q else np.ones(len(fields))
        if m.metric not in _DISTANCE_METRICS and m.metric not in _SIMILARITY_METRICS:
            raise UnsupportedFeatureException(f"clustering metric {m.metric!r}")
        for cf in self.compare:
            if cf not in ("absDiff", "gaussSim", "delta", "equal"):
                raise UnsupportedFeatureException(f"compareFunction {cf!r}")
        self.metric = m.metric
        self.p = m.minkowski_p
        self.kind_distance = m.measure_kind == "distance"

    def feature_matrix(self, cols: Columns) -> np.ndarray:
        return np.stack([cols.get(f) for f in self.fields], axis=1) if self.fields else np.zeros((cols.n, 0))

    def distances(self, X: np.ndarray) -> np.ndarray:
        """``[n, K]`` distance (or similarity) matrix, float64."""
        n, F = X.shape
        K = self.centers.shape[0]
        # bounded [rows, K, F] blocks: every row's distances are independent, so the chunked
        # result is bit-identical (a 256-centre x 128-field model no longer builds GBs at once)
        chunk = max(1, (1 << 22) // max(1, K * F))
        if n > chunk:
            return np.concatenate([self.distances(X[i:i + chunk]) for i in range(0, n, chunk)], axis=0)
        miss = np.isnan(X)
        if self.metric in _SIMILARITY_METRICS:
            return self._binary_similarity(X)
        diff = X[:, None, :] - self.centers[None, :, :]
        cfs = np.asarray(self.compare, dtype=object)
        kinds = set(self.compare)
        comp = np.empty((n, K, F)) if len(kinds) > 1 else None
        for cf in kinds:  # the same element-wise formulas as one field at a time, per group
            cols = slice(None) if comp is None else np.flatnonzero(cfs == cf)
            d = diff[:, :, cols]
            if cf == "absDiff":
                v = np.abs(d)
            elif cf == "gaussSim":
                s = self.scales[cols]
                v = np.exp(-np.log(2.0) * d * d / (s * s))
            elif cf == "delta":
                v = (d != 0).astype(np.float64)
            else:  # equal
                v = (d == 0).astype(np.float64)
            if comp is None:
                comp = np.ascontiguousarray(v, dtype=np.float64)
            else:
                comp[:, :, cols] = v
        comp[np.broadcast_to(miss[:, None, :], comp.shape)] = 0.0
        w = self.weights[None, None, :]
        if self.metric == "squaredEuclidean":
            s = np.sum(w * comp * comp, axis=2)
        elif self.metric == "euclidean":
            s = np.sum(w * comp * comp, axis=2)
        elif self.metric == "cityBlock":
            s = np.sum(w * comp, axis=2)
        elif self.metric == "minkowski":
            s = np.sum(w * np.power(comp, self.p), axis=2)
        else:  # chebychev
            s = np.max(w * comp, axis=2)
        if self.metric != "chebychev":
            q = self.missing_weights
            present_q = np.sum(np.where(miss, 0.0, q[None, :]), axis=1)
            with np.errstate(divide="ignore", invalid="ignore"):
                adj = np.where(present_q > 0, q.sum() / present_q, NAN)
            s = s * adj[:, None]
        if self.metric == "euclidean":
            s = np.sqrt(s)
        elif self.metric == "minkowski":
            s = np.power(s, 1.0 / self.p)
        return s

    def _binary_similarity(self, X: np.ndarray) -> np.ndarray:
        x = (X[:, None, :] == 1.0)
        y = (self.centers[None, :, :] == 1.0)
        a11 = np.sum(x & y, axis=2).astype(np.float64)
        a10 = np.sum(x & ~y, axis=2).astype(np.float64)
        a01 = np.sum(~x & y, axis=2).astype(np.float64)
        a00 = np.sum(~x & ~y, axis=2).astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.metric == "simpleMatching":
                return (a11 + a00) / (a11 + a10 + a01 + a00)
            if self.metric == "jaccard":
                return a11 / (a11 + a10 + a01)
            if self.metric == "tanimoto":
                return (a11 + a00) / (a11 + 2 * (a10 + a01) + a00)
        raise UnsupportedFeatureException("binarySimilarity needs explicit parameters")

    def _evaluate(self, cols: Columns) -> ModelResult:
        X = self.feature_matrix(cols)
        D = self.distances(X)
        all_missing = np.all(np.isnan(X), axis=1)
        Dz = np.where(np.isnan(D), np.inf if self.kind_distance else -np.inf, D)
        idx = np.argmin(Dz, axis=1) if self.kind_distance else np.argmax(Dz, axis=1)
        valid = ~all_missing & np.isfinite(Dz[np.arange(len(idx)), idx])
        aff = D[np.arange(len(idx)), idx]
        return ModelResult(
            kind="clustering",
            value=np.where(valid, idx.astype(np.float64), NAN),
            valid=valid,
            entity_ids=self.entity_ids,
            affinity=aff,
            entity_affinities=D,
        )
