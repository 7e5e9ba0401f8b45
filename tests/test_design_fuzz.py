"""Randomized RegressionModels through the design-matrix lowering (`runtime/design.py`): random
tables of numeric predictors (exponents 1-3), categorical predictors on the string field ``color``,
interaction terms (2-3 fields, repeats allowed), intercepts, and a random normalizationMethod —
regression links, or classification with 2-5 tables (softmax, simplemax, the binary rule, one
element-wise link per table). CPU: the derive program's numpy twin + the dense tables reproduce
the float64 oracle; GPU: the DerivedPlan (derive kernel → linear kernel) vs the oracle."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.bench.synth import mixed_records
from flink_jpmml_amd.runtime.compiled import CompiledPmml

NS = "http://www.dmg.org/PMML-4_4"
F = 4
LEVELS = ("red", "green", "blue")
REG_NORMS = ["none", "logit", "exp", "probit", "cloglog", "loglog", "cauchit"]
CLS_NORMS = ["softmax", "simplemax", "logit", "probit", "cloglog", "none"]


def _table(rng, category=None) -> str:
    tc = f' targetCategory="{category}"' if category is not None else ""
    out = [f'<RegressionTable intercept="{rng.normal() * 0.5:.4f}"{tc}>']
    for j in rng.permutation(F)[: int(rng.integers(1, F + 1))]:
        e = int(rng.choice([1, 1, 2, 3]))
        ex = f' exponent="{e}"' if e != 1 else ""
        out.append(f'<NumericPredictor name="f{j}"{ex} coefficient="{rng.normal() * 0.4:.4f}"/>')
    for v in rng.permutation(LEVELS)[: int(rng.integers(0, 3))]:
        out.append(f'<CategoricalPredictor name="color" value="{v}" coefficient="{rng.normal():.4f}"/>')
    for _ in range(int(rng.integers(0, 3))):
        fields = [f"f{int(k)}" for k in rng.integers(0, F, int(rng.integers(2, 4)))]
        out.append(f'<PredictorTerm coefficient="{rng.normal() * 0.3:.4f}">'
                   + "".join(f'<FieldRef field="{f}"/>' for f in fields) + '</PredictorTerm>')
    out.append('</RegressionTable>')
    return "".join(out)


def _doc(seed: int) -> tuple:
    rng = np.random.default_rng(5000 + seed)
    classes = int(rng.choice([0, 0, 2, 3, 5]))
    if classes:
        norm = str(rng.choice(CLS_NORMS))
        if norm == "simplemax":
            classes = max(classes, 2)
        cats = [str(k) for k in range(classes)]
        target = ('<DataField name="y" optype="categorical" dataType="string">'
                  + "".join(f'<Value value="{c}"/>' for c in cats) + '</DataField>')
        tables = "".join(_table(rng, c) for c in cats)
        fn = "classification"
    else:
        norm = str(rng.choice(REG_NORMS))
        target = '<DataField name="y" optype="continuous" dataType="double"/>'
        tables = _table(rng)
        fn = "regression"
    doc = (f'<PMML version="4.4" xmlns="{NS}"><DataDictionary>'
           + "".join(f'<DataField name="f{j}" optype="continuous" dataType="double"/>' for j in range(F))
           + '<DataField name="color" optype="categorical" dataType="string">'
           + "".join(f'<Value value="{v}"/>' for v in LEVELS) + '</DataField>' + target + '</DataDictionary>'
           f'<RegressionModel functionName="{fn}" normalizationMethod="{norm}"><MiningSchema>'
           '<MiningField name="y" usageType="target"/>'
           + "".join(f'<MiningField name="f{j}"/>' for j in range(F))
           + '<MiningField name="color"/></MiningSchema>' + tables + '</RegressionModel></PMML>')
    return doc, classes, norm


def _inputs(n: int, seed: int) -> np.ndarray:
    _, X = mixed_records(n, F, seed=seed, missing_rate=0.04)
    return X


@pytest.mark.parametrize("seed", range(40))
def test_design_twin_matches_oracle(seed):
    from flink_jpmml_amd.runtime.derive import emulate
    from flink_jpmml_amd.runtime.design import design_layout
    from flink_jpmml_amd.runtime.plans import NotLowerable, lowering_dry_run

    doc, classes, norm = _doc(seed)
    c = CompiledPmml.from_string(doc)
    try:
        layout, dense = design_layout(c)
    except NotLowerable:
        pytest.skip("dense table (no design program needed)")
    X = _inputs(2000, seed)
    P, ok = c.prepare(X)
    D = emulate(layout.program, P).astype(np.float64)
    W, b = dense.dense_weights()
    res = dense.finish(D @ W + b, ok & ~np.isnan(D).any(axis=1))
    full = c.result(X)
    assert (res.valid == full.valid).all(), (seed, norm)
    v = res.valid
    if classes:
        assert (res.value[v] == full.value[v]).mean() > 0.995
        # fp32 design columns: simplemax over a near-zero table sum amplifies rounding, so compare
        # relatively and allow a handful of such rows
        a, b = res.probs[v], full.probs[v]
        assert (np.abs(a - b) > 1e-4 * np.maximum(1.0, np.abs(b))).mean() < 0.002, (seed, norm)
    else:
        np.testing.assert_allclose(res.value[v], full.value[v], rtol=1e-4, atol=1e-4)
    with lowering_dry_run():
        c.plan("cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(40, 12))
def test_design_plans_on_gpu(gpu, seed):
    doc, classes, norm = _doc(seed)
    c = CompiledPmml.from_string(doc)
    plan = c.plan(gpu)
    X = _inputs(20000, seed + 100)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), (seed, norm, int((v != vref).sum()))
    if not v.any():
        return
    if classes:
        assert (s[v] == ref[v]).mean() > 0.995, (seed, norm)
    else:
        scale = np.maximum(1.0, np.abs(ref[v]))
        assert (np.abs(s[v] - ref[v]) <= 2e-4 * scale).mean() > 0.999, (seed, norm)
