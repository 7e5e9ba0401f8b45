"""AssociationModel (association rules) — float64 host oracle.

The reference evaluates every PMML model through JPMML (`S/api/PmmlModel.scala:159-160`) and keeps
only the first *target* field (`S/api/PmmlModel.scala:167-174`); an AssociationModel has no target
field, so ``predict`` yields ``EmptyScore`` for every record there and here, while loading the model
succeeds. What such a model computes — the rules whose itemsets match a record's basket — is exposed
through ``ruleValue`` / ``entityId`` output fields (``PmmlModel.predict_with_outputs``), following
the PMML 4.x association-rule semantics:

* a record's basket is the set of item values of its active fields (categorical codes decoded to
  their values, numbers written as in the document: ``3`` for 3.0);
* ``algorithm``: ``recommendation`` — the antecedent is in the basket; ``exclusiveRecommendation``
  (default) — and no consequent item is; ``ruleAssociation`` — antecedent and consequent are;
* the matching rules are ordered by ``rankBasis`` (confidence by default; support, lift, leverage,
  affinity) in ``rankOrder`` (descending by default; ties keep document order) and the ``rank``-th
  (1-based) is reported as its ``ruleFeature``: antecedent / consequent (the item value, or
  ``{a,b}`` for several items), ``rule`` (``{a}->{b}``), ``ruleId``, or one of the rule's measures.

No device kernel: set matching over a handful of rules per basket is host work (SURVEY §2.8 lists
no association op); the device path scores such models with the NullScorer (no target)."""

from __future__ import annotations

import math
from typing import List, Optional

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema
from .base import ModelEvaluator, ModelResult

_MEASURES = ("support", "confidence", "lift", "leverage", "affinity")


def _fmt(v) -> Optional[str]:
    if v is None:
        return None
    if isinstance(v, float):
        if math.isnan(v):
            return None
        if v.is_integer():
            return str(int(v))
        return repr(v)
    return str(v)


class AssociationEvaluator(ModelEvaluator):
    kind = "association"

    def __init__(self, model: ir.AssociationModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.kind = "association"
        self.sets = {sid: frozenset(model.items[i] for i in ids) for sid, ids in model.itemsets.items()}
        self.rules: List[ir.AssociationRule] = list(model.rules)

    def _evaluate(self, cols: Columns) -> ModelResult:
        n = cols.n
        decoded = []
        for f in self.active_fields:
            col = cols.get(f)
            decoded.append([_fmt(self.schema.decode(f, float(v))) for v in col])
        baskets = [frozenset(d[i] for d in decoded if d[i] is not None) for i in range(n)]
        res = ModelResult("association", np.full(n, NAN), np.zeros(n, dtype=bool))
        res.extra["baskets"] = baskets
        return res

    # ------------------------------------------------------------------ rule outputs
    def _matching(self, basket: frozenset, algorithm: str) -> List[int]:
        out = []
        for k, r in enumerate(self.rules):
            a, c = self.sets[r.antecedent], self.sets[r.consequent]
            if not a <= basket:
                continue
            # PMML: the rule is excluded when its whole consequent is already in the basket
            # (a consequent that only partly overlaps is still recommended)
            if algorithm == "exclusiveRecommendation" and c <= basket:
                continue
            if algorithm == "ruleAssociation" and not c <= basket:
                continue
            out.append(k)
        return out

    def _ranked(self, basket: frozenset, of: ir.OutputField) -> Optional[ir.AssociationRule]:
        if of.algorithm not in ("recommendation", "exclusiveRecommendation", "ruleAssociation"):
            raise UnsupportedFeatureException(f"association algorithm {of.algorithm!r}")
        basis = of.rank_basis if of.rank_basis in _MEASURES else "confidence"
        ks = self._matching(basket, of.algorithm)
        sign = -1.0 if of.rank_order != "ascending" else 1.0

        def key(k):
            v = getattr(self.rules[k], basis)
            return (sign * (v if v is not None else -math.inf), k)  # stable: document order on ties

        ks.sort(key=key)
        r = of.rank if of.rank and of.rank > 0 else 1
        return self.rules[ks[r - 1]] if len(ks) >= r else None

    def _items_text(self, sid: str) -> str:
        vals = sorted(self.sets[sid])
        return vals[0] if len(vals) == 1 else "{" + ",".join(vals) + "}"

    def _rule_value(self, rule: ir.AssociationRule, feature: str):
        if feature == "antecedent":
            return self._items_text(rule.antecedent)
        if feature == "consequent":
            return self._items_text(rule.consequent)
        if feature == "rule":
            a = ",".join(sorted(self.sets[rule.antecedent]))
            c = ",".join(sorted(self.sets[rule.consequent]))
            return "{" + a + "}->{" + c + "}"
        if feature == "ruleId":
            return rule.rule_id if rule.rule_id is not None else str(self.rules.index(rule) + 1)
        if feature in _MEASURES:
            v = getattr(rule, feature)
            return NAN if v is None else float(v)
        raise UnsupportedFeatureException(f"association ruleFeature {feature!r}")

    def _output_column(self, of: ir.OutputField, cols: Columns, res: ModelResult, n: int) -> np.ndarray:
        if of.feature not in ("ruleValue", "entityId"):
            return super()._output_column(of, cols, res, n)
        feature = "ruleId" if of.feature == "entityId" else of.rule_feature
        baskets = res.extra["baskets"]
        col = np.full(n, NAN)
        numeric = feature in _MEASURES
        if not numeric:
            self.schema.types.setdefault(of.name, "string")
        for i, b in enumerate(baskets):
            rule = self._ranked(b, of)
            if rule is None:
                continue
            v = self._rule_value(rule, feature)
            col[i] = v if numeric else self.schema.lookup(of.name, v)
        return col
