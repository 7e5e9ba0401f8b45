"""MiningModel (ensembles / model chains): GBDT, random forests, calibrated chains.

``Segmentation/@multipleModelMethod``:

* regression: ``sum``, ``average``, ``weightedAverage``, ``median``, ``weightedMedian``, ``max``,
  ``min``;
* classification: ``majorityVote``, ``weightedMajorityVote``, ``average``, ``weightedAverage``,
  ``max``, ``median``;
* any: ``selectFirst`` (first segment whose predicate is TRUE), ``modelChain`` (segments run in
  order, each one's ``<Output>`` fields feed the next; the last applicable segment is the result).

``missingPredictionTreatment``: ``returnMissing``/``continue`` make the aggregate missing when a
segment yields no prediction; ``skipSegment`` ignores such segments.
"""

from __future__ import annotations

from typing import List

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema, eval_predicate
from ..pmml.mathcontext import is_float
from .base import ModelEvaluator, ModelResult


class MiningEvaluator(ModelEvaluator):
    def __init__(self, model: ir.MiningModel, schema: FieldSchema):
        super().__init__(model, schema)
        from .registry import make_evaluator  # circular

        self.mm = model
        self.method = model.multiple_model_method
        self.segments = model.segments
        self.sub = [make_evaluator(s.model, schema) for s in model.segments]
        self.weights = np.array([s.weight for s in model.segments], dtype=np.float64)
        if self.kind == "classification":
            cats = self.classification_categories()
            seen = set(cats)
            for ev in self.sub:
                for c in getattr(ev, "categories", None) or []:
                    if c not in seen:
                        cats.append(c)
                        seen.add(c)
            self.categories = cats
        else:
            self.categories = None

    # ------------------------------------------------------------------ native forest pass
    _REGRESS_METHODS = ("sum", "weightedSum", "average", "weightedAverage", "max", "min", "median",
                        "weightedMedian")

    def native_forest(self):
        """One :class:`~flink_jpmml_amd.models.native_tree.ForestProgram` over every segment when
        this is a regression ensemble of plain trees (True segment predicates, regression trees
        without outputs / local transformations / targets): the whole segment loop is then one
        native call producing the ``[rows, segments]`` value matrix ``_regress`` aggregates.
        None otherwise (built once)."""
        prog = getattr(self, "_native", False)
        if prog is False:
            prog = None
            from .tree import TreeEvaluator

            if self.kind == "regression" and self.method in self._REGRESS_METHODS and self.sub and all(
                    isinstance(seg.predicate, ir.TruePredicate) and type(ev) is TreeEvaluator
                    and ev.kind == "regression" and not ev.model.output and not ev.model.local_transformations
                    and ev.target is None and not getattr(ev, "value_fields", None)
                    for seg, ev in zip(self.segments, self.sub)):
                from .native_tree import forest_program

                prog = forest_program(self.sub, [ev.node_value for ev in self.sub])
            self._native = prog
        return prog

    def native_vote(self):
        """``(ForestProgram, class table, node offsets, weights)`` when this is a (weighted)
        majority vote over plain classification trees (True segment predicates, no outputs / local
        transformations, no mixture missing strategies): the whole vote is then one native leaf
        walk plus a bincount, instead of one Python tree evaluation per segment. None otherwise."""
        vote = getattr(self, "_native_vote", False)
        if vote is False:
            vote = None
            from .tree import TreeEvaluator

            if self.kind == "classification" and self.method in ("majorityVote", "weightedMajorityVote") and self.sub \
                    and all(isinstance(seg.predicate, ir.TruePredicate) and type(ev) is TreeEvaluator
                            and ev.kind == "classification" and not ev.model.output
                            and not ev.model.local_transformations and not getattr(ev, "value_fields", None)
                            and ev.tree.missing_value_strategy not in ("weightedConfidence", "aggregateNodes")
                            for seg, ev in zip(self.segments, self.sub)):
                from .native_tree import forest_program

                cats = self.categories
                tabs, offs, off = [], [], 0
                for ev in self.sub:
                    idx_map = np.array([cats.index(c) for c in ev.categories], dtype=np.int64)
                    lab = np.asarray(ev.node_label, dtype=np.float64)
                    ok = ~np.isnan(lab)
                    tabs.append(np.where(ok, idx_map[np.where(ok, lab, 0).astype(np.int64)], -1))
                    offs.append(off)
                    off += len(lab)
                prog = forest_program(self.sub, [np.zeros(len(ev.node_label)) for ev in self.sub])
                if prog is not None:
                    # the class of every node in the program's global numbering (tree t at roots[t])
                    roots = np.asarray(prog.roots, dtype=np.int64)
                    gcls = np.full(int(sum(len(t) for t in tabs)), -1, dtype=np.int32)
                    for t, tab in enumerate(tabs):
                        gcls[roots[t]:roots[t] + len(tab)] = tab
                    vote = (prog, np.concatenate(tabs).astype(np.int64), np.asarray(offs, dtype=np.int64),
                            np.asarray(self.weights, dtype=np.float64), gcls)
            self._native_vote = vote
        return vote

    def _vote_native(self, L: np.ndarray, glab: np.ndarray, offs: np.ndarray, w: np.ndarray) -> ModelResult:
        """``_classify`` for a (weighted) majority vote from the ``[T, n]`` leaf matrix: the same
        per-(row, class) additions in tree order (bincount over the tree-major entries), so the
        vote shares are bit-identical to the per-segment loop."""
        T, n = L.shape
        C = len(self.categories)
        G = np.where(L >= 0, L + offs[:, None], -1)
        lab = np.where(G >= 0, glab[np.maximum(G, 0)], -1)
        use = lab >= 0
        ww = w if self.method == "weightedMajorityVote" else np.ones(T)
        rows = np.broadcast_to(np.arange(n, dtype=np.int64), (T, n))
        wts = np.broadcast_to(ww[:, None], (T, n))[use]
        acc = np.bincount((rows * C + lab)[use], weights=wts, minlength=n * C).reshape(n, C)
        wsum = np.bincount(rows[use], weights=wts, minlength=n)
        return self._class_result(acc, wsum, use.sum(axis=0), ~use.all(axis=0))

    def _evaluate(self, cols: Columns) -> ModelResult:
        n = cols.n
        method = self.method
        vote = self.native_vote() if n else None
        if vote is not None:
            try:
                X = vote[0].matrix(cols)
            except Exception:  # noqa: BLE001 - a field the segments reference cannot be prepared
                X = None
            if X is not None:
                prog, glab, offs, w, gcls = vote
                ww = w if method == "weightedMajorityVote" else np.ones(len(w))
                from ..native import fastpath

                if hasattr(fastpath(), "forest_votes"):
                    acc, wsum, count, anymiss = prog.votes(X, gcls, ww, len(self.categories))
                    return self._class_result(acc, wsum, count, anymiss)
                return self._vote_native(prog.leaves(X), glab, offs, w)  # (an older _fastpath build)
        prog = self.native_forest() if n else None
        if prog is not None:
            try:
                X = prog.matrix(cols)
            except Exception:  # noqa: BLE001 - a field the segments reference cannot be prepared
                X = None
            if X is not None:
                if method in ("sum", "weightedSum", "average", "weightedAverage") and not is_float(self.mm) \
                        and self.mm.missing_prediction_treatment != "skipSegment":
                    # every segment applies: a row is valid iff no tree is null, and the value is
                    # _regress's np.sum over the row (the native sum reproduces its pairwise order)
                    weighted = method in ("weightedSum", "weightedAverage")
                    out = prog.sums(X, self.weights if weighted else None)
                    with np.errstate(invalid="ignore", divide="ignore"):
                        if method == "average":
                            out = out / len(self.sub)
                        elif method == "weightedAverage":
                            out = out / np.sum(self.weights)
                    return ModelResult("regression", out, np.isfinite(out))
                V = prog.values(X)
                return self._regress_matrix(V, np.ones(V.shape, dtype=bool))
        results: List[ModelResult] = []
        applies: List[np.ndarray] = []
        chain = method == "modelChain"
        for seg, ev in zip(self.segments, self.sub):
            t, _u = eval_predicate(seg.predicate, cols)
            if method == "selectFirst" and results:
                taken = np.zeros(n, dtype=bool)
                for a in applies:
                    taken |= a
                if taken.all():
                    break
            r = ev.evaluate(cols)
            if chain or ev.model.output:
                outs = ev.compute_outputs(cols, r)
                # rows the segment does not apply to must not see its outputs
                if not t.all():
                    for k, v in outs.items():
                        cols.set(k, np.where(t, v, NAN))
            results.append(r)
            applies.append(t)
        if not results:
            return ModelResult(self.kind, np.full(n, NAN), np.zeros(n, dtype=bool), categories=self.categories)
        if method in ("modelChain", "selectFirst"):
            return self._select(results, applies, last=(method == "modelChain"))
        if self.kind == "classification":
            return self._classify(results, applies)
        return self._regress(results, applies)

    # ------------------------------------------------------------------ selection
    def _select(self, results: List[ModelResult], applies: List[np.ndarray], last: bool) -> ModelResult:
        n = results[0].n
        chosen = np.full(n, -1)
        order = range(len(results) - 1, -1, -1) if last else range(len(results))
        for i in order:
            chosen = np.where((chosen < 0) & applies[i], i, chosen)
        final = results[-1] if last else results[0]
        kind = final.kind
        value = np.full(n, NAN)
        valid = np.zeros(n, dtype=bool)
        cats = final.categories if kind == "classification" else None
        probs = np.full((n, len(cats)), NAN) if cats is not None and final.probs is not None else None
        ent = [None] * n
        for i, r in enumerate(results):
            m = chosen == i
            if not m.any():
                continue
            if kind == "classification" and r.kind == "classification" and r.categories != cats:
                # remap to the final segment's category order
                remap = np.array([cats.index(c) if c in cats else -1 for c in r.categories], dtype=np.float64)
                v = np.where(r.valid, remap[np.where(r.valid, r.value, 0).astype(int)], NAN)
                value[m] = v[m]
            else:
                value[m] = r.value[m]
            valid[m] = r.valid[m]
            if probs is not None and r.probs is not None and r.probs.shape[1] == probs.shape[1]:
                probs[m] = r.probs[m]
            el = r.extra.get("entity_labels")
            if el is not None:
                for j in np.nonzero(m)[0]:
                    ent[j] = el[j]
        res = ModelResult(kind, value, valid & ~np.isnan(value), categories=cats, probs=probs,
                          entity_ids=final.entity_ids, affinity=None)
        if kind == "clustering":
            res.affinity = final.affinity
        res.extra["entity_labels"] = ent
        return res

    # ------------------------------------------------------------------ regression
    def _regress(self, results: List[ModelResult], applies: List[np.ndarray]) -> ModelResult:
        V = np.stack([np.where(r.valid, r.value, NAN) for r in results], axis=1)
        A = np.stack(applies, axis=1)
        return self._regress_matrix(V, A)

    def _regress_matrix(self, V: np.ndarray, A: np.ndarray) -> ModelResult:
        """Aggregate the ``[rows, segments]`` values ``V`` (NaN = no prediction) of the segments
        that apply (``A``)."""
        W = np.broadcast_to(self.weights[None, :], V.shape)
        miss = np.isnan(V) & A
        skip = self.mm.missing_prediction_treatment == "skipSegment"
        use = A & ~np.isnan(V)
        method = self.method
        with np.errstate(invalid="ignore", divide="ignore"):
            Vz = np.where(use, V, 0.0)
            if is_float(self.mm) and method in ("sum", "weightedSum", "average", "weightedAverage"):
                out = _float_aggregate(method, Vz, W, use)
            elif method == "sum":
                out = np.sum(Vz, axis=1)
            elif method == "weightedSum":  # PMML 4.4: Σ weight · value over the used segments
                out = np.sum(Vz * W, axis=1)
            elif method == "average":
                out = np.sum(Vz, axis=1) / np.sum(use, axis=1)
            elif method == "weightedAverage":
                out = np.sum(Vz * W, axis=1) / np.sum(np.where(use, W, 0.0), axis=1)
            elif method in ("max", "min"):
                fill = -np.inf if method == "max" else np.inf
                Vf = np.where(use, V, fill)
                out = Vf.max(axis=1) if method == "max" else Vf.min(axis=1)
            elif method == "median":
                out = np.nanmedian(np.where(use, V, NAN), axis=1)
            elif method == "weightedMedian":
                out = _weighted_median(V, W, use)
            else:
                raise UnsupportedFeatureException(f"multipleModelMethod {method!r} for regression")
        valid = np.any(use, axis=1)
        if not skip:
            valid &= ~np.any(miss, axis=1)
        out = np.where(valid, out, NAN)
        return ModelResult("regression", out, valid & np.isfinite(out))

    # ------------------------------------------------------------------ classification
    def _classify(self, results: List[ModelResult], applies: List[np.ndarray]) -> ModelResult:
        cats = self.categories
        C = len(cats)
        n = results[0].n
        method = self.method
        acc = np.zeros((n, C))
        wsum = np.zeros(n)
        anymiss = np.zeros(n, dtype=bool)
        count = np.zeros(n)
        for r, a, w in zip(results, applies, self.weights):
            use = a & r.valid
            anymiss |= a & ~r.valid
            if r.kind != "classification":
                raise UnsupportedFeatureException("classification ensemble over non-classification segments")
            idx_map = np.array([cats.index(c) for c in r.categories])
            if method in ("majorityVote", "weightedMajorityVote"):
                lab = idx_map[np.where(use, r.value, 0).astype(int)]
                ww = w if method == "weightedMajorityVote" else 1.0
                np.add.at(acc, (np.nonzero(use)[0], lab[use]), ww)
                wsum += np.where(use, ww, 0.0)
            else:
                P = np.zeros((n, C))
                P[:, idx_map] = np.nan_to_num(r.probs) if r.probs is not None else 0.0
                if method in ("average", "weightedAverage"):
                    ww = w if method == "weightedAverage" else 1.0
                    acc += np.where(use[:, None], P * ww, 0.0)
                    wsum += np.where(use, ww, 0.0)
                elif method == "max":
                    acc = np.where(use[:, None], np.maximum(acc, P), acc)
                elif method == "median":
                    acc += 0  # handled below
                else:
                    raise UnsupportedFeatureException(f"multipleModelMethod {method!r} for classification")
            count += use
        if method == "median":
            stack = []
            for r, a in zip(results, applies):
                idx_map = np.array([cats.index(c) for c in r.categories])
                P = np.full((n, C), NAN)
                P[:, idx_map] = r.probs
                P[~(a & r.valid)] = NAN
                stack.append(P)
            acc = np.nanmedian(np.stack(stack, axis=0), axis=0)
        return self._class_result(acc, wsum, count, anymiss)

    def _class_result(self, acc: np.ndarray, wsum: np.ndarray, count: np.ndarray, anymiss: np.ndarray) -> ModelResult:
        method, cats = self.method, self.categories
        with np.errstate(invalid="ignore", divide="ignore"):
            if method in ("majorityVote", "weightedMajorityVote", "average", "weightedAverage"):
                probs = acc / wsum[:, None]
            else:
                probs = acc
        valid = count > 0
        if self.mm.missing_prediction_treatment != "skipSegment":
            valid &= ~anymiss
        lab = np.argmax(np.nan_to_num(probs, nan=-1.0), axis=1).astype(np.float64)
        return ModelResult("classification", np.where(valid, lab, NAN), valid, categories=cats,
                           probs=np.where(valid[:, None], probs, NAN))


def _float_aggregate(method: str, Vz: np.ndarray, W: np.ndarray, use: np.ndarray) -> np.ndarray:
    """``x-mathContext="float"``: the segment values summed in float32, in segment order."""
    acc = np.zeros(Vz.shape[0], dtype=np.float32)
    wsum = np.zeros(Vz.shape[0], dtype=np.float32)
    for j in range(Vz.shape[1]):
        v = Vz[:, j].astype(np.float32)
        weighted = method in ("weightedAverage", "weightedSum")
        w = W[:, j].astype(np.float32) if weighted else np.float32(1.0)
        acc = acc + (w * v if weighted else v)
        wsum = wsum + np.where(use[:, j], w, np.float32(0.0))
    if method in ("sum", "weightedSum"):
        return acc.astype(np.float64)
    return (acc / wsum).astype(np.float64)


def _weighted_median(V: np.ndarray, W: np.ndarray, use: np.ndarray) -> np.ndarray:
    out = np.full(V.shape[0], NAN)
    for i in range(V.shape[0]):
        v = V[i, use[i]]
        w = W[i, use[i]]
        if v.size == 0:
            continue
        o = np.argsort(v, kind="stable")
        cw = np.cumsum(w[o])
        out[i] = v[o][np.searchsorted(cw, 0.5 * cw[-1])]
    return out
