"""NearestNeighborModel (k-NN over inline ``TrainingInstances``).

Distances use the ClusteringModel comparison machinery (``ComparisonMeasure`` metric ×
``compareFunction`` × ``fieldWeight``, missing inputs skipped with the Σq/Σq_present rescale) with
the training instances as centres; the ``k`` nearest (ties: lower instance index) are aggregated:

* classification: ``majorityVote`` / ``weightedMajorityVote`` (weight ``1 / (d + threshold)``);
  ties between classes go to the class whose best member ranks first;
* regression: ``average`` / ``median`` / ``weightedAverage``.

JPMML scores it per record (`S/api/PmmlModel.scala:159-160`). Device: ``k == 1`` *is* a
ClusteringModel whose centres are the instances and whose entity labels are their targets, so it
runs on ``cluster.hip`` (the MFMA distance expansion for many instances); ``k > 1`` (and any model
with a ``Targets`` rescale) runs on ``knn.hip`` (register top-k + aggregation, ``KnnPlan``).
Parity unpinned (no JPMML here): follows the PMML 4.4 specification text.
"""

from __future__ import annotations

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from .base import ModelResult
from .clustering import ClusteringEvaluator

_ROW_BLOCK = 2048


def knn_as_clustering(m: ir.NearestNeighborModel, schema: FieldSchema) -> ir.ClusteringModel:
    fields = [ir.ClusteringField(k.field, k.weight, k.compare_function) for k in m.inputs]
    centers = []
    for r in m.rows:
        c = []
        for k in m.inputs:
            col = m.instance_fields.get(k.field, k.field)
            v = r.get(col)
            if v is None or v == "":
                raise UnsupportedFeatureException("training instance with a missing input value")
            c.append(float(schema.lookup(k.field, v)))
        centers.append(c)
    tgt = m.mining_schema.targets[0].name if m.mining_schema.targets else None
    tcol = m.instance_fields.get(tgt, tgt) if tgt else None
    clusters = [ir.Cluster(None, r.get(tcol) if tcol else str(i + 1), c) for i, (r, c) in enumerate(zip(m.rows, centers))]
    return ir.ClusteringModel(element="ClusteringModel", model_name=m.model_name, function_name="clustering",
                              mining_schema=m.mining_schema, output=[], targets=[], local_transformations=[],
                              measure_kind=m.measure_kind, metric=m.metric, minkowski_p=m.minkowski_p,
                              compare_function=m.compare_function, fields=fields, clusters=clusters)


class NearestNeighborEvaluator(ClusteringEvaluator):
    def __init__(self, model: ir.NearestNeighborModel, schema: FieldSchema):
        if not model.mining_schema.targets:
            raise UnsupportedFeatureException("NearestNeighborModel without a target field")
        super().__init__(knn_as_clustering(model, schema), schema)
        self.knn = model
        self.model = model  # outputs / targets / transformations of the original element
        self.target = next((t for t in model.targets if t.field is None or t.field == self.target_field), None)
        self.k = max(1, int(model.k))
        self.kind = "classification" if model.function_name == "classification" else "regression"
        self.targets = list(self.entity_ids)  # instance target strings
        if self.kind == "classification":
            cats = self.classification_categories()
            for t in self.targets:
                if t not in cats:
                    cats.append(t)
            self.categories = cats
            self.inst_class = np.array([cats.index(t) for t in self.targets])
        else:
            self.categories = None
            self.inst_value = np.array([float(t) for t in self.targets])

    def _evaluate(self, cols: Columns) -> ModelResult:
        X = self.feature_matrix(cols)
        n = X.shape[0]
        k = min(self.k, len(self.targets))
        nn = np.zeros((n, k), dtype=np.int64)
        dist = np.zeros((n, k))
        for r0 in range(0, n, _ROW_BLOCK):
            D = self.distances(X[r0: r0 + _ROW_BLOCK])
            D = np.where(np.isnan(D), np.inf, D) if self.kind_distance else np.where(np.isnan(D), np.inf, -D)
            o = np.argsort(D, axis=1, kind="stable")[:, :k]
            nn[r0: r0 + _ROW_BLOCK] = o
            dist[r0: r0 + _ROW_BLOCK] = np.take_along_axis(D, o, axis=1)
        valid = np.isfinite(dist).all(axis=1) & ~np.all(np.isnan(X), axis=1)
        m = self.knn
        if self.kind == "classification":
            C = len(self.categories)
            votes = np.zeros((n, C))
            first = np.full((n, C), k, dtype=np.int64)
            w = _weights(dist, m.threshold) if m.categorical_method == "weightedMajorityVote" else np.ones_like(dist)
            if m.categorical_method not in ("majorityVote", "weightedMajorityVote"):
                raise UnsupportedFeatureException(f"categoricalScoringMethod {m.categorical_method!r}")
            rows = np.arange(n)
            for j in range(k):
                c = self.inst_class[nn[:, j]]
                votes[rows, c] += np.where(np.isfinite(w[:, j]), w[:, j], 0.0)
                first[rows, c] = np.minimum(first[rows, c], j)
            best = votes.max(axis=1, keepdims=True)
            lab = np.argmin(np.where(votes == best, first, k + 1), axis=1).astype(np.float64)
            with np.errstate(invalid="ignore"):
                probs = votes / votes.sum(axis=1, keepdims=True)
            return ModelResult("classification", np.where(valid, lab, NAN), valid, categories=self.categories,
                               probs=np.where(valid[:, None], probs, NAN))
        y = self.inst_value[nn]
        meth = m.continuous_method
        if meth == "average":
            v = y.mean(axis=1)
        elif meth == "median":
            v = np.median(y, axis=1)
        elif meth == "weightedAverage":
            w = _weights(dist, m.threshold)
            with np.errstate(invalid="ignore"):  # rows without neighbours (all fields missing): NaN
                v = (w * y).sum(axis=1) / w.sum(axis=1)
        else:
            raise UnsupportedFeatureException(f"continuousScoringMethod {meth!r}")
        return ModelResult("regression", np.where(valid, v, NAN), valid & np.isfinite(v))


def _weights(dist: np.ndarray, threshold: float) -> np.ndarray:
    """Neighbour weights ``1 / (|d| + threshold)`` of the weighted scoring methods. A zero
    denominator (an exact match with ``threshold = 0``) would make the weighted average inf / inf;
    its limit as the distance goes to 0 is the exact matches alone, equally weighted — so a row
    with any exact match weighs those 1 and the others 0 (the kernel applies the same rule)."""
    with np.errstate(divide="ignore"):
        w = 1.0 / (np.abs(dist) + threshold)
    exact = ~np.isfinite(w) & ~np.isnan(w)
    if exact.any():
        rows = exact.any(axis=1)
        w[rows] = exact[rows].astype(np.float64)
    return w
