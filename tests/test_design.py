"""Design-matrix lowering of RegressionModel (categorical predictors, terms, exponents) and
GeneralRegressionModel (covariates, factors, interactions; identity / log / logit / power links,
multinomial logistic) — ``runtime/design.py``.

CPU: the design derive program (numpy twin :func:`derive.emulate`) + the dense tables reproduce the
float64 oracle; GPU: the DerivedPlan (derive kernel → linear kernel) against the oracle.
"""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import glm_pmml, mixed_records, naive_bayes_pmml, regression_design_pmml
from flink_jpmml_amd.runtime.compiled import CompiledPmml

CASES = {
    "reg": lambda: regression_design_pmml(),
    "reg-logit": lambda: regression_design_pmml(normalization="logit"),
    "reg-softmax": lambda: regression_design_pmml(classes=3, normalization="softmax"),
    "reg-binary": lambda: regression_design_pmml(classes=2, normalization="logit"),
    # > 2 tables with an element-wise link (one-vs-rest logistic exports): p_k = link(y_k), argmax
    "reg-ovr-logit": lambda: regression_design_pmml(classes=3, normalization="logit"),
    "reg-ovr-none": lambda: regression_design_pmml(classes=4, normalization="none", seed=2),
    "reg-ovr-probit": lambda: regression_design_pmml(classes=3, normalization="probit", seed=3),
    "reg-ovr-cloglog": lambda: regression_design_pmml(classes=5, normalization="cloglog", seed=4),
    "reg-ovr-exp": lambda: regression_design_pmml(classes=3, normalization="exp", seed=5),
    "glm-log": lambda: glm_pmml(link="log"),
    "glm-logit": lambda: glm_pmml(link="logit"),
    "glm-identity": lambda: glm_pmml(link="identity"),
    "glm-power0": lambda: glm_pmml(link="power"),
    "glm-general-linear": lambda: glm_pmml(model_type="generalLinear"),
    "glm-multinomial": lambda: glm_pmml(model_type="multinomialLogistic"),
    "glm-ordinal-logit": lambda: glm_pmml(model_type="ordinalMultinomial", link="logit", classes=4),
    "glm-ordinal-probit": lambda: glm_pmml(model_type="ordinalMultinomial", link="probit", seed=2),
    "glm-ordinal-cloglog": lambda: glm_pmml(model_type="ordinalMultinomial", link="cloglog", classes=5, seed=3),
    "glm-ordinal-loglog": lambda: glm_pmml(model_type="ordinalMultinomial", link="loglog", seed=4),
    "glm-ordinal-cauchit": lambda: glm_pmml(model_type="ordinalMultinomial", link="cauchit", seed=5),
    # binomial GLM (classification generalizedLinear): P(event) = F(η), the reference 1 - P;
    # reference listed first (mirrored link in the lowering), last, or by default
    "glm-binomial-logit-first": lambda: glm_pmml(link="logit", binomial="first", seed=6),
    "glm-binomial-probit-last": lambda: glm_pmml(link="probit", binomial="last", seed=7),
    "glm-binomial-cloglog-first": lambda: glm_pmml(link="cloglog", binomial="first", seed=8, event_cells=False),
    "glm-binomial-loglog-default": lambda: glm_pmml(link="loglog", binomial="default", seed=9),
    "glm-binomial-loglog-first": lambda: glm_pmml(link="loglog", binomial="first", seed=10),
    "glm-binomial-identity-first": lambda: glm_pmml(link="identity", binomial="first", seed=11),
    "naive-bayes": lambda: naive_bayes_pmml(),
    "naive-bayes-2": lambda: naive_bayes_pmml(classes=2, seed=3),
    # BayesInput with its own DerivedField (Discretize bins keyed PairCounts) / the same bins as a
    # LocalTransformations field
    "naive-bayes-discretized": lambda: naive_bayes_pmml(seed=4, discretized="inline"),
    "naive-bayes-local-bins": lambda: naive_bayes_pmml(seed=4, discretized="local"),
}


def _data(c, n=3000, missing=0.05, seed=0):
    _, X = mixed_records(n, len(c.active_fields) - 1, seed=seed, missing_rate=missing)
    return X


@pytest.mark.parametrize("name", list(CASES))
def test_design_program_matches_oracle(name):
    from flink_jpmml_amd.runtime.derive import emulate
    from flink_jpmml_amd.runtime.design import design_layout, needs_design

    c = CompiledPmml.from_string(CASES[name]())
    assert needs_design(c.evaluator)
    layout, dense = design_layout(c)
    assert dense.is_dense_linear() and layout.program is not None
    assert list(layout.columns) == list(dense.numeric_fields)
    X = _data(c)
    P, ok = c.prepare(X)
    D = emulate(layout.program, P).astype(np.float64)
    W, b = dense.dense_weights()
    res = dense.finish(D @ W + b, ok & ~np.isnan(D).any(axis=1))
    ref, vref = c.score_matrix_oracle(X)
    assert (res.valid == vref).all()
    if res.kind == "classification":  # numeric category labels: the score is the label's value
        labels = np.array([float(k) for k in res.categories])
        assert (labels[res.value[vref].astype(int)] == ref[vref]).mean() > 0.999
        full = c.result(X)  # class probabilities in category order (mirrored binomial tables too)
        assert list(full.categories) == list(res.categories)
        np.testing.assert_allclose(res.probs[vref], full.probs[vref], rtol=1e-5, atol=1e-6)  # fp32 design columns
    else:
        assert np.allclose(res.value[vref], ref[vref], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("ref", ["first", "last", "default"])
@pytest.mark.parametrize("event_cells", [True, False])
def test_binomial_glm_oracle_by_hand(ref, event_cells):
    """P("1") = logistic(offset + Σ β·design), P("0") (the reference) = 1 − P("1"); the label is
    the larger one."""
    c = CompiledPmml.from_string(glm_pmml(link="logit", binomial=ref, event_cells=event_cells, seed=3))
    ev = c.evaluator
    assert ev.binomial_roles() == ("0", "1")
    gm = ev.gm
    beta = {p: b for p, _, b in gm.p_cells}
    _, X = mixed_records(40, 3, seed=12, missing_rate=0.1)
    res = c.result(X)
    cats = ev.categories
    levels = c.schema.data_fields["color"].values
    for r in range(len(X)):
        f0, f1, f2, code = X[r]
        if np.isnan([f0, f1, f2]).any():
            assert not res.valid[r]
            continue
        color = levels[int(code)] if not np.isnan(code) else None
        eta = gm.offset_value + beta["p0"] + beta["p1"] * f0 + beta["p2"] * f1 ** 2 + beta["p3"] * f2
        eta += beta["pc1"] * (color == "red") + beta["pc2"] * (color == "green") + beta["px"] * (color == "blue") * f0
        p_yes = 1.0 / (1.0 + np.exp(-eta))
        assert res.valid[r]
        assert np.isclose(res.probs[r, cats.index("1")], p_yes, rtol=1e-12)
        assert np.isclose(res.probs[r, cats.index("0")], 1.0 - p_yes, rtol=1e-12)
        assert res.value[r] == (cats.index("1") if p_yes > 0.5 else cats.index("0"))


def test_ordinal_glm_oracle_by_hand():
    """eta_j = offset + cut_j + shared slopes, P(Y<=j) = logistic(eta_j), P(j) = differences."""
    c = CompiledPmml.from_string(glm_pmml(model_type="ordinalMultinomial", link="logit", classes=4, seed=7))
    gm = c.evaluator.gm
    _, X = mixed_records(6, 3, seed=11, missing_rate=0.1)
    beta = {(p, tc): b for p, tc, b in gm.p_cells}
    res = c.result(X)
    for r in range(len(X)):
        f0, f1, f2, code = X[r]
        if np.isnan([f0, f1, f2]).any():
            assert not res.valid[r]
            continue
        lvl = ["red", "green", "blue"][int(code)] if not np.isnan(code) else None
        cols = {"p1": f0, "p2": f1 ** 2, "p3": f2, "pc1": float(lvl == "red"), "pc2": float(lvl == "green"),
                "px": float(lvl == "blue") * f0}
        shared = 0.25 + sum(beta[(p, None)] * v for p, v in cols.items())
        cum = [1 / (1 + np.exp(-(beta[("p0", str(j))] + shared))) for j in range(3)] + [1.0]
        probs = np.diff(cum, prepend=0.0)
        np.testing.assert_allclose(res.probs[r], probs, rtol=1e-12)
        assert res.value[r] == float(np.argmax(probs))


def test_glm_oracle_semantics():
    """Hand check of the GLM oracle on one record: eta = offset + Σ beta·design, log link."""
    c = CompiledPmml.from_string(glm_pmml(link="log"))
    gm = c.evaluator.gm
    beta = {p: b for p, _, b in gm.p_cells}
    x = np.array([[0.5, -1.0, 2.0, 2.0]])  # color code 2 = blue
    eta = gm.offset_value + beta["p0"] + beta["p1"] * 0.5 + beta["p2"] * 1.0 + beta["p3"] * 2.0 + beta["px"] * 0.5
    s, v = c.score_matrix_oracle(x)
    assert v[0] and np.isclose(s[0], np.exp(eta))


def test_naive_bayes_oracle_by_hand():
    """One record, spec formula: n_j · Π N(x_i; μ_ij, σ²_ij) · P(color | j), normalised."""
    import math

    c = CompiledPmml.from_string(naive_bayes_pmml(seed=1))
    nb = c.model
    x = {"f0": 0.3, "f1": -1.2, "f2": 0.0, "f3": 2.0}
    post = []
    for k in ("0", "1", "2"):
        p = nb.target_counts[k]
        for inp in nb.inputs[:4]:
            mu, var = inp.gaussian[k]
            p *= math.exp(-(x[inp.field] - mu) ** 2 / (2 * var)) / math.sqrt(2 * math.pi * var)
        cnt = nb.inputs[4].pair_counts["blue"][k]
        p *= (cnt / nb.target_counts[k]) if cnt > 0 else nb.threshold
        post.append(p)
    post = np.array(post) / sum(post)
    res = c.result(np.array([[0.3, -1.2, 0.0, 2.0, 2.0]]))  # color code 2 = blue
    assert np.allclose(res.probs[0], post, rtol=1e-9)
    assert res.value[0] == np.argmax(post)


def test_design_not_lowerable_power_link():
    from flink_jpmml_amd.runtime.design import design_layout
    from flink_jpmml_amd.runtime.plans import NotLowerable

    txt = glm_pmml(link="power").replace('linkParameter="0"', 'linkParameter="0.5"')
    with pytest.raises(NotLowerable):
        design_layout(CompiledPmml.from_string(txt))


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_design_plan_on_gpu(gpu, name):
    from flink_jpmml_amd.runtime.derive import DerivedPlan
    from flink_jpmml_amd.runtime.plans import LinearPlan

    c = CompiledPmml.from_string(CASES[name]())
    plan = c.plan(gpu)
    assert isinstance(plan, DerivedPlan) and isinstance(plan.inner, LinearPlan)
    X = _data(c, n=20000, seed=1)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if plan.inner.table is not None:
        assert (s[v] == ref[v]).mean() > 0.999
    else:
        assert np.allclose(s[v], ref[v], rtol=1e-4, atol=1e-4)


def test_naive_bayes_inline_discretization():
    """A BayesInput's own DerivedField scores exactly like the same bins as a LocalTransformations
    field, and the bin edges follow the Interval closures (-0.5 is "mid", just below is "low")."""
    inline = CompiledPmml.from_string(naive_bayes_pmml(seed=4, discretized="inline"))
    local = CompiledPmml.from_string(naive_bayes_pmml(seed=4, discretized="local"))
    _, X = mixed_records(3000, 4, seed=6, missing_rate=0.05)
    ra, rb = inline.result(X), local.result(X)
    assert (ra.valid == rb.valid).all() and ra.valid.any()
    np.testing.assert_array_equal(ra.probs[ra.valid], rb.probs[rb.valid])
    row = X[:1].copy()
    row[0, :3] = 0.1
    row[0, 4] = 0.0

    def probs(v):
        r = row.copy()
        r[0, 3] = v
        return inline.result(r).probs[0]

    np.testing.assert_array_equal(probs(-0.5), probs(0.49))       # both "mid"
    np.testing.assert_array_equal(probs(-0.6), probs(-3.0))       # both "low"
    assert not np.array_equal(probs(-0.5), probs(np.nextafter(-0.5, -1.0)))  # mid | low edge
    assert not np.array_equal(probs(0.5), probs(0.49))            # high | mid edge
