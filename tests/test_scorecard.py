"""Scorecard and RuleSetModel (``models/scorecard.py``): load-time rewrite into the tree IR.

Parity unpinned: JPMML is not available here, so the oracle is checked against an independent
per-record re-implementation of the PMML 4.4 specification text (below), and the GPU against the
oracle.
"""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import mixed_records, ruleset_pmml, scorecard_pmml
from flink_jpmml_amd.pmml import ir
from flink_jpmml_amd.runtime.compiled import CompiledPmml

LEVELS = ["red", "green", "blue"]


def _pred(p, rec):
    """Per-record three-valued predicate (True / False / None = unknown), spec semantics."""
    if isinstance(p, ir.TruePredicate):
        return True
    if isinstance(p, ir.FalsePredicate):
        return False
    if isinstance(p, ir.SimplePredicate):
        x = rec.get(p.field)
        if p.operator == "isMissing":
            return x is None
        if p.operator == "isNotMissing":
            return x is not None
        if x is None:
            return None
        v = p.value if p.field == "color" else float(p.value)
        return {"lessThan": lambda: x < v, "greaterOrEqual": lambda: x >= v, "greaterThan": lambda: x > v,
                "lessOrEqual": lambda: x <= v, "equal": lambda: x == v, "notEqual": lambda: x != v}[p.operator]()
    if isinstance(p, ir.SimpleSetPredicate):
        x = rec.get(p.field)
        if x is None:
            return None
        return (x in p.values) == (p.boolean_operator == "isIn")
    if isinstance(p, ir.CompoundPredicate):
        vals = [_pred(q, rec) for q in p.predicates]
        assert p.boolean_operator == "and"
        if any(v is False for v in vals):
            return False
        return None if any(v is None for v in vals) else True
    raise AssertionError(p)


def _scorecard_ref(sc, rec):
    total = sc.initial_score
    for ch in sc.characteristics:
        hit = next((a for a in ch.attributes if _pred(a.predicate, rec) is True), None)
        if hit is None:
            return None
        total += hit.partial_score
    return total


@pytest.mark.parametrize("seed", [0, 1])
def test_scorecard_matches_spec(seed):
    txt = scorecard_pmml(seed=seed)
    c = CompiledPmml.from_string(txt)
    sc = c.model
    assert isinstance(sc, ir.Scorecard)
    recs, X = mixed_records(600, 4, seed=seed, missing_rate=0.08)
    s, v = c.score_matrix_oracle(X)
    for r, rec in enumerate(recs):
        ref = _scorecard_ref(sc, rec)
        assert v[r] == (ref is not None)
        if ref is not None:
            assert abs(s[r] - ref) < 1e-9
    assert 0 < v.mean() < 1  # some rows hit an unmatched characteristic


def test_scorecard_reason_codes():
    c = CompiledPmml.from_string(scorecard_pmml(seed=3))
    sc = c.model
    recs, X = mixed_records(50, 4, seed=4)
    res = c.result(X)
    rc = res.extra["reason_codes"]
    for r, rec in enumerate(recs):
        acc = {}
        for ch in sc.characteristics:
            a = next(a for a in ch.attributes if _pred(a.predicate, rec) is True)
            base = ch.baseline_score if ch.baseline_score is not None else sc.baseline_score
            code = a.reason_code or ch.reason_code
            acc[code] = acc.get(code, 0.0) + (base - a.partial_score)
        ranked = [k for k, _ in sorted(acc.items(), key=lambda kv: -kv[1])]
        assert rc[r] == ranked
    _, outs = c.evaluate_prepared(c.prepare(X)[0])
    assert set(outs) == {"RC1", "RC2"}


def _ruleset_ref(rs, rec):
    flat = []

    def walk(rules, guards):
        for r in rules:
            if isinstance(r, ir.CompoundRule):
                walk(r.rules, guards + [r.predicate])
            else:
                flat.append((r, guards + [r.predicate]))

    walk(rs.rules, [])
    fired = [(i, r) for i, (r, ps) in enumerate(flat) if all(_pred(p, rec) is True for p in ps)]
    if not fired:
        return rs.default_score
    if rs.criterion == "firstHit":
        return fired[0][1].score
    if rs.criterion == "weightedMax":
        best = max(r.weight for _, r in fired)
        return next(r.score for _, r in fired if r.weight == best)
    tot, first = {}, {}
    for i, r in fired:
        tot[r.score] = tot.get(r.score, 0.0) + r.weight
        first.setdefault(r.score, i)
    best = max(tot.values())
    return min((first[k], k) for k, t in tot.items() if t == best)[1]


@pytest.mark.parametrize("criterion", ["firstHit", "weightedMax", "weightedSum"])
@pytest.mark.parametrize("default", [True, False])
def test_ruleset_matches_spec(criterion, default):
    c = CompiledPmml.from_string(ruleset_pmml(criterion=criterion, default=default, seed=5, n_rules=10))
    recs, X = mixed_records(800, 4, seed=6, missing_rate=0.05)
    s, v = c.score_matrix_oracle(X)
    for r, rec in enumerate(recs):
        ref = _ruleset_ref(c.model, rec)
        assert v[r] == (ref is not None)
        if ref is not None:
            assert s[r] == float(ref)
    if not default:
        assert not v.all()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["scorecard", "firstHit", "weightedMax"])
def test_scorecard_ruleset_on_gpu(gpu, kind):
    from flink_jpmml_amd.runtime.plans import TreePlan

    txt = scorecard_pmml(seed=2) if kind == "scorecard" else ruleset_pmml(criterion=kind, seed=7, default=False)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    inner = getattr(plan, "inner", plan)
    assert isinstance(inner, TreePlan)
    _, X = mixed_records(20_000, 4, seed=8, missing_rate=0.05)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if kind == "scorecard":
        assert np.allclose(s[v], ref[v], rtol=1e-5, atol=1e-4)
    else:
        assert (s[v] == ref[v]).all()


@pytest.mark.parametrize("kind", ["scorecard", "firstHit", "weightedMax"])
def test_general_layout_emulation(kind):
    """CPU twin of the device path: GENERAL-layout packing + numpy walk == oracle."""
    from flink_jpmml_amd.runtime.derive import FieldView, plan_field_layout
    from flink_jpmml_amd.runtime.general_tree import emulate_general, lower_general_tree, pack_general
    from flink_jpmml_amd.runtime.plans import ensemble_spec

    txt = scorecard_pmml(seed=2) if kind == "scorecard" else ruleset_pmml(criterion=kind, seed=7, default=False)
    c = CompiledPmml.from_string(txt)
    layout = plan_field_layout(c, allow_alias=True)
    assert layout.program is None
    view = FieldView(c, layout, prepared=False)
    spec = ensemble_spec(view, lower=lower_general_tree)
    packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
    _, X = mixed_records(400, 4, seed=8, missing_rate=0.05)
    P, _ = c.prepare(X)
    acc = emulate_general(packed, P.astype(np.float32), spec.P, len(spec.trees))
    ref, vref = c.score_matrix_oracle(X)
    ok = ~np.isnan(acc).any(axis=1)
    assert (ok == vref).all()
    e = spec.epi
    if kind == "scorecard":
        assert np.allclose(e["a"] * acc[ok, 0] + e["b"], ref[ok], atol=1e-4)
    else:
        lab = np.array([float(x) for x in spec.labels])[np.argmax(acc[ok], axis=1)]
        assert (lab == ref[ok]).all()


def _with_complex_score(txt: str) -> tuple:
    """ch1's first attribute (f1 < t) scores the expression 2 * f1 + 3 instead of its constant."""
    import re

    m = re.search(r'<Attribute partialScore="([^"]+)">(<SimplePredicate field="f1" operator="lessThan" '
                  r'value="([^"]+)"/>)</Attribute>', txt)
    assert m is not None
    cps = ('<ComplexPartialScore><Apply function="+"><Apply function="*"><FieldRef field="f1"/>'
           '<Constant>2</Constant></Apply><Constant>3</Constant></Apply></ComplexPartialScore>')
    out = txt[:m.start()] + f'<Attribute partialScore="{m.group(1)}">{m.group(2)}{cps}</Attribute>' + txt[m.end():]
    return out, float(m.group(1)), float(m.group(3))


@pytest.mark.parametrize("seed", [0, 1])
def test_complex_partial_score(seed):
    """ComplexPartialScore (precedence over partialScore): the attribute's points are the expression
    on the record; everything else equals the constant scorecard. The MiningModel rewrite (a leaf
    reading a synthetic derived field) equals the direct formulation bit for bit."""
    from flink_jpmml_amd.models.scorecard import ComplexScorecardEvaluator, ScorecardEvaluator

    base = scorecard_pmml(seed=seed)
    txt, const, thr = _with_complex_score(base)
    c0, c1 = CompiledPmml.from_string(base), CompiledPmml.from_string(txt)
    assert isinstance(c1.evaluator, ScorecardEvaluator)
    _, X = mixed_records(800, 4, seed=seed + 5, missing_rate=0.08)
    s0, v0 = c0.score_matrix_oracle(X)
    s1, v1 = c1.score_matrix_oracle(X)
    assert (v0 == v1).all() and v1.any()
    hit = X[:, 1] < thr
    assert hit[v1].any() and (~hit[v1]).any()
    np.testing.assert_allclose(s1[v1 & ~hit], s0[v1 & ~hit], rtol=0, atol=1e-9)
    np.testing.assert_allclose(s1[v1 & hit], (s0 - const + 2 * X[:, 1] + 3)[v1 & hit], rtol=0, atol=1e-9)
    # the direct formulation
    direct = ComplexScorecardEvaluator(c1.evaluator.scorecard, c1.schema)
    P, ok = c1.prepare(X)
    rd = direct.evaluate(c1.columns(P))
    np.testing.assert_array_equal(rd.valid & ok, v1)
    np.testing.assert_allclose(rd.value[v1], s1[v1], rtol=0, atol=1e-9)
    # reason codes use the expression's points too
    res = c1.result(X[:50])
    assert len(res.extra["reason_codes"]) == 50


@pytest.mark.parametrize("seed", [0, 1])
def test_complex_partial_score_lowers_to_the_general_layout(seed):
    """Round 6: the synthetic derived field is a derive-pass column and the
    GENERAL kernel adds it to the leaf (``vcol``); the CPU twin equals the oracle."""
    from flink_jpmml_amd.runtime.derive import FieldView, plan_field_layout
    from flink_jpmml_amd.runtime.general_tree import emulate_general, lower_general_tree, pack_general
    from flink_jpmml_amd.runtime.plans import compile_plan, ensemble_spec, lowering_dry_run

    txt, _, _ = _with_complex_score(scorecard_pmml(seed=seed))
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        plan = compile_plan(c, "cpu")
    assert type(plan).__name__ == "DerivedPlan"
    layout = plan_field_layout(c, allow_alias=True)
    assert layout.program is not None
    view = FieldView(c, layout, prepared=True)
    spec = ensemble_spec(view, lower=lower_general_tree)
    packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
    assert packed["vcol"] is not None and (packed["vcol"] >= 0).sum() == 1
    _, X = mixed_records(600, 4, seed=seed + 9, missing_rate=0.08)
    P, _ = c.prepare(X)
    # the derive pass's columns: the active inputs, then the derived fields the layout computes
    cols = c.columns(P)
    model = c.evaluator.model
    child = cols.child(model.local_transformations)
    Xk = np.stack([child.get(name) for name in layout.columns], axis=1)
    acc = emulate_general(packed, Xk.astype(np.float32), spec.P, len(spec.trees))
    ref, vref = c.score_matrix_oracle(X)
    ok = ~np.isnan(acc).any(axis=1)
    assert (ok == vref).all()
    e = spec.epi
    assert np.allclose(e["a"] * acc[ok, 0] + e["b"], ref[ok], atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_complex_partial_score_on_gpu(gpu, seed):
    """ComplexPartialScore scorecards on the device (derive pass + GENERAL kernel leaf column)."""
    from flink_jpmml_amd.runtime.plans import TreePlan

    txt, _, _ = _with_complex_score(scorecard_pmml(seed=seed))
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    assert isinstance(getattr(plan, "inner", plan), TreePlan)
    _, X = mixed_records(20_000, 4, seed=seed + 3, missing_rate=0.08)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and v.any()
    assert np.allclose(s[v], ref[v], rtol=1e-5, atol=1e-4)
