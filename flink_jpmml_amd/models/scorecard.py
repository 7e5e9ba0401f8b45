"""Scorecard and RuleSetModel.

Both are evaluated by JPMML per record like every other model (`S/api/PmmlModel.scala:159-160`).
Here they are *rewritten* once, at load time, into the tree IR, so the float64 oracle and the GPU
kernels are the existing ones:

* **Scorecard** = ``initialScore + Σ_characteristics partialScore(first attribute whose predicate
  is TRUE)`` — a ``MiningModel`` ``sum`` of one multiway ``TreeModel`` per characteristic (root →
  one child per attribute, document order) plus a root-only tree holding ``initialScore``. An
  UNKNOWN predicate (missing input) does not match (``missingValueStrategy="none"``); a
  characteristic without a matching attribute has no partial score, which makes the whole score
  missing (``returnNullPrediction`` + ``sum``'s missing rule) → ``EmptyScore``. Multiway trees lower
  to the GENERAL tree layout (``tree.hip::tree_general_kernel``). An Attribute with a
  ``ComplexPartialScore`` (an expression over the record, taking precedence over ``partialScore``)
  becomes a leaf that reads its value per record from a synthetic DerivedField (``__cps_<i>_<j>``,
  the expression, in the rewrite's LocalTransformations): the device's derive pass computes the
  column and the GENERAL tree kernel adds it (``tree.hip`` ``vcol``); a missing expression value
  voids the score. :class:`ComplexScorecardEvaluator` is the direct formulation kept for the
  tests. Reason codes
  (``useReasonCodes``, ``pointsBelow`` / ``pointsAbove``) are host outputs.
* **RuleSetModel** ``firstHit`` = a one-level ``TreeModel``: the (flattened) rules are the root's
  children in document order, a ``CompoundRule``'s predicate AND-ed into its rules; the
  ``defaultScore`` sits on the root (``returnLastPrediction``). ``weightedMax`` is ``firstHit`` over
  the rules stably sorted by descending weight. ``weightedSum`` (score with the largest weight sum
  over all firing rules) is host-only.

Parity: no JPMML in this environment — the semantics follow the PMML 4.4 specification text;
marked "parity unpinned" in ``tests/test_scorecard.py``.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema, eval_expression, eval_predicate
from .base import ModelEvaluator, ModelResult
from .mining import MiningEvaluator
from .tree import TreeEvaluator


def _common(m: ir.Model, element: str, **over) -> dict:
    d = dict(element=element, model_name=m.model_name, function_name=m.function_name,
             mining_schema=m.mining_schema, output=m.output, targets=m.targets,
             local_transformations=m.local_transformations, is_scorable=m.is_scorable,
             algorithm_name=m.algorithm_name)
    d.update(over)
    return d


def _segment_tree(sc: ir.Model, root: ir.Node, **kw) -> ir.TreeModel:
    return ir.TreeModel(**_common(sc, "TreeModel", function_name="regression", output=[], targets=[],
                                  local_transformations=[]), root=root, **kw)


def complex_field(i: int, j: int) -> str:
    """Name of the synthetic DerivedField holding characteristic i / attribute j's
    ComplexPartialScore expression."""
    return f"__cps_{i}_{j}"


def scorecard_as_mining(sc: ir.Scorecard) -> ir.MiningModel:
    segs = [ir.Segment("initialScore", 1.0, ir.TruePredicate(),
                       _segment_tree(sc, ir.Node("initialScore", repr(float(sc.initial_score)), ir.TruePredicate())))]
    extra: List[ir.DerivedField] = []
    for i, ch in enumerate(sc.characteristics):
        kids = []
        for j, a in enumerate(ch.attributes):
            if a.complex_score is not None:
                # a ComplexPartialScore: the leaf reads its value per record from a synthetic
                # DerivedField of the scorecard's scope (a missing value voids the score)
                name = complex_field(i, j)
                extra.append(ir.DerivedField(name, "continuous", "double", a.complex_score))
                kids.append(ir.Node(f"c{i}a{j}", "0", a.predicate, value_field=name))
                continue
            if a.partial_score is None:
                raise UnsupportedFeatureException("Scorecard Attribute without partialScore")
            kids.append(ir.Node(f"c{i}a{j}", repr(float(a.partial_score)), a.predicate))
        root = ir.Node(f"c{i}", None, ir.TruePredicate(), children=kids)
        tree = _segment_tree(sc, root, missing_value_strategy="none", no_true_child_strategy="returnNullPrediction")
        segs.append(ir.Segment(ch.name or f"c{i}", 1.0, ir.TruePredicate(), tree))
    common = _common(sc, "MiningModel", function_name="regression")
    if extra:
        common["local_transformations"] = list(common["local_transformations"] or []) + extra
    return ir.MiningModel(**common, multiple_model_method="sum", segments=segs,
                          missing_prediction_treatment="returnMissing")


def _picks(sc: ir.Scorecard, cols: Columns) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Per characteristic: the first attribute whose predicate is TRUE (-1: none) and its partial
    score per row (NaN without a match; a ComplexPartialScore evaluated on the record)."""
    n = cols.n
    out = []
    for ch in sc.characteristics:
        pick = np.full(n, -1)
        for j, a in enumerate(ch.attributes):
            t, _ = eval_predicate(a.predicate, cols)
            pick = np.where((pick < 0) & t, j, pick)
        partial = np.full(n, NAN)
        for j, a in enumerate(ch.attributes):
            sel = pick == j
            if not sel.any():
                continue
            if a.complex_score is not None:
                partial[sel] = eval_expression(a.complex_score, cols)[sel]
            elif a.partial_score is not None:
                partial[sel] = a.partial_score
            else:
                raise UnsupportedFeatureException("Scorecard Attribute without partialScore")
        out.append((pick, partial))
    return out


class _ReasonCodes:
    """Reason-code outputs shared by both scorecard evaluators."""

    def _reason_codes(self, cols: Columns) -> List[List[str]]:
        """Per row: reason codes ranked by their summed point difference to the baseline
        (``pointsBelow``: baseline − partial; ``pointsAbove``: partial − baseline), ties in
        characteristic order."""
        sc = self.scorecard
        n = cols.n
        diffs: List[Tuple[np.ndarray, np.ndarray, List[Optional[str]]]] = []
        for ch, (pick, partial) in zip(sc.characteristics, _picks(sc, cols)):
            base = ch.baseline_score if ch.baseline_score is not None else sc.baseline_score
            if base is None:
                raise UnsupportedFeatureException("reason codes need a baselineScore")
            d = (base - partial) if sc.reason_code_algorithm == "pointsBelow" else (partial - base)
            codes = [a.reason_code or ch.reason_code for a in ch.attributes]
            diffs.append((pick, d, codes))
        out: List[List[str]] = []
        for r in range(n):
            acc: dict = {}
            for pick, d, codes in diffs:
                if pick[r] >= 0 and codes[pick[r]] is not None:
                    acc[codes[pick[r]]] = acc.get(codes[pick[r]], 0.0) + float(d[r])
            out.append([c for c, _ in sorted(acc.items(), key=lambda kv: -kv[1])])
        return out

    def _output_column(self, of: ir.OutputField, cols: Columns, res: ModelResult, n: int) -> np.ndarray:
        if of.feature == "reasonCode":
            rc = res.extra.get("reason_codes")
            if rc is None:
                return np.full(n, NAN)
            k = max(1, int(of.rank)) - 1
            return self._encode_label(of.name, [r[k] if len(r) > k and v else None for r, v in zip(rc, res.valid)])
        return super()._output_column(of, cols, res, n)

    def _with_reason_codes(self, res: ModelResult, cols: Columns) -> ModelResult:
        if self.scorecard.use_reason_codes and any(of.feature == "reasonCode" for of in self.model.output):
            res.extra["reason_codes"] = self._reason_codes(cols)
        return res


class ScorecardEvaluator(_ReasonCodes, MiningEvaluator):
    def __init__(self, model: ir.Scorecard, schema: FieldSchema):
        if model.function_name not in ("regression", ""):
            raise UnsupportedFeatureException(f"Scorecard functionName {model.function_name!r}")
        self.scorecard = model
        super().__init__(scorecard_as_mining(model), schema)

    def _evaluate(self, cols: Columns) -> ModelResult:
        return self._with_reason_codes(super()._evaluate(cols), cols)


class ComplexScorecardEvaluator(_ReasonCodes, ModelEvaluator):
    """Scorecards with ``ComplexPartialScore`` attributes: ``initialScore + Σ partial`` evaluated
    directly (no constant-leaf tree form, so no device plan: ``compile_plan`` falls back to host)."""

    def __init__(self, model: ir.Scorecard, schema: FieldSchema):
        if model.function_name not in ("regression", ""):
            raise UnsupportedFeatureException(f"Scorecard functionName {model.function_name!r}")
        super().__init__(model, schema)
        self.scorecard = model
        self.categories = None

    def _evaluate(self, cols: Columns) -> ModelResult:
        total = np.full(cols.n, float(self.scorecard.initial_score))
        for _, partial in _picks(self.scorecard, cols):
            total = total + partial  # no matching attribute / missing expression value -> NaN
        ok = np.isfinite(total)
        return self._with_reason_codes(ModelResult("regression", np.where(ok, total, NAN), ok), cols)


def make_scorecard_evaluator(model: ir.Scorecard, schema: FieldSchema) -> ModelEvaluator:
    """Every scorecard — ComplexPartialScore attributes included (leaves reading a synthetic
    derived field, so the device lowers them too) — runs as its MiningModel rewrite;
    :class:`ComplexScorecardEvaluator` stays the direct formulation the tests check it against."""
    return ScorecardEvaluator(model, schema)


# --------------------------------------------------------------------------- rule sets


def _flatten(rules: List[object], guard: List[ir.Predicate]) -> List[Tuple[ir.SimpleRule, ir.Predicate]]:
    out = []
    for r in rules:
        if isinstance(r, ir.CompoundRule):
            out.extend(_flatten(r.rules, guard + [r.predicate]))
        else:
            p = r.predicate if not guard else ir.CompoundPredicate("and", guard + [r.predicate])
            out.append((r, p))
    return out


def ruleset_as_tree(rs: ir.RuleSetModel) -> ir.TreeModel:
    rules = _flatten(rs.rules, [])
    if rs.criterion == "weightedMax":
        rules = sorted(rules, key=lambda rp: -rp[0].weight)  # stable: document order on ties
    elif rs.criterion != "firstHit":
        raise UnsupportedFeatureException(f"RuleSet criterion {rs.criterion!r} has no tree form")
    kids = [ir.Node(r.id or f"rule{i}", r.score, p, distributions=list(r.distributions))
            for i, (r, p) in enumerate(rules)]
    root = ir.Node("default", rs.default_score, ir.TruePredicate(), children=kids)
    return ir.TreeModel(**_common(rs, "TreeModel"), root=root, missing_value_strategy="none",
                        no_true_child_strategy="returnLastPrediction" if rs.default_score is not None
                        else "returnNullPrediction")


class RuleSetEvaluator(TreeEvaluator):
    """``firstHit`` / ``weightedMax`` rule sets through the tree oracle (and GENERAL kernel)."""

    def __init__(self, model: ir.RuleSetModel, schema: FieldSchema):
        self.ruleset = model
        super().__init__(ruleset_as_tree(model), schema)


class WeightedSumRuleSetEvaluator(ModelEvaluator):
    """``weightedSum``: every firing rule votes its weight for its score; the largest total wins
    (ties: the score that fired first in document order). Host only."""

    def __init__(self, model: ir.RuleSetModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.rules = _flatten(model.rules, [])
        cats = self.classification_categories() if self.kind == "classification" else []
        for r, _ in self.rules:
            if r.score not in cats:
                cats.append(r.score)
        if model.default_score is not None and model.default_score not in cats:
            cats.append(model.default_score)
        self.categories = cats

    def _evaluate(self, cols: Columns) -> ModelResult:
        n = cols.n
        C = len(self.categories)
        tot = np.zeros((n, C))
        first = np.full((n, C), np.inf)
        for i, (r, p) in enumerate(self.rules):
            t, _ = eval_predicate(p, cols)
            k = self.categories.index(r.score)
            tot[:, k] += np.where(t, r.weight, 0.0)
            first[:, k] = np.where(t & np.isinf(first[:, k]), i, first[:, k])
        fired = np.isfinite(first).any(axis=1)
        # largest weight sum; ties -> earliest first firing
        tot_f = np.where(np.isfinite(first), tot, -np.inf)
        cand = tot_f == tot_f.max(axis=1, keepdims=True)
        lab = np.argmin(np.where(cand, first, np.inf), axis=1).astype(np.float64)
        rs: ir.RuleSetModel = self.model
        if rs.default_score is not None:
            lab = np.where(fired, lab, float(self.categories.index(rs.default_score)))
            ok = np.ones(n, dtype=bool)
        else:
            ok = fired
        kind = "classification" if self.kind == "classification" else "regression"
        if kind == "regression":
            vals = np.array([float(c) for c in self.categories])
            return ModelResult(kind, np.where(ok, vals[lab.astype(int)], NAN), ok)
        probs = np.zeros((n, C))
        probs[np.arange(n), lab.astype(int)] = 1.0
        return ModelResult(kind, np.where(ok, lab, NAN), ok, categories=self.categories,
                           probs=np.where(ok[:, None], probs, NAN))


def make_ruleset_evaluator(model: ir.RuleSetModel, schema: FieldSchema) -> ModelEvaluator:
    if model.criterion == "weightedSum":
        return WeightedSumRuleSetEvaluator(model, schema)
    return RuleSetEvaluator(model, schema)
