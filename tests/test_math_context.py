"""``x-mathContext="float"`` (jpmml-xgboost / jpmml-lightgbm exports): float32 literals and float32
accumulation (``pmml/mathcontext.py``). Parity unpinned (no JPMML here): the checks pin the
documented intent — split decisions of a float32 evaluator, float32 segment sums — and that the
device plans agree with that oracle."""

import re

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
from flink_jpmml_amd.pmml import flat, parser
from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _decimal_thresholds(txt: str) -> str:
    """Rewrite every split value as a 6-digit decimal (mostly NOT float32-representable)."""
    return re.sub(r'value="(-?[0-9.eE+-]+)"', lambda m: f'value="{float(m.group(1)):.6g}"', txt)


def _float_ctx(txt: str) -> str:
    for el in ("MiningModel", "TreeModel", "RegressionModel"):
        txt = txt.replace(f"<{el} ", f'<{el} x-mathContext="float" ')
    return txt


def _edge_inputs(c, n=4000, seed=0):
    """Rows whose split features sit exactly on float32(threshold) — where float and double
    evaluation of ``x < t`` / ``x >= t`` disagree for non-representable thresholds."""
    X = stream_matrix(n, c.n_features, seed=seed).astype(np.float64)
    thr = {}
    for m in parser.iter_models(c.doc):
        if hasattr(m, "flat") and m.root is not None:
            stack = [m.root]
            while stack:
                nd = stack.pop()
                p = nd.predicate
                if getattr(p, "value", None) is not None and getattr(p, "field", None) in c.active_fields:
                    thr.setdefault(c.active_fields.index(p.field), []).append(float(p.value))
                stack.extend(nd.children)
    rng = np.random.default_rng(seed)
    for j, ts in thr.items():
        pick = rng.random(n) < 0.5
        X[pick, j] = np.float32(rng.choice(ts, pick.sum()))
    return X.astype(np.float32)


@pytest.fixture(params=["dom", "scanner"])
def reader(request, monkeypatch):
    if request.param == "scanner":
        monkeypatch.setattr(flat, "SCAN_MIN_BYTES", 0)
    return request.param


def test_float_context_parsed_and_inherited(reader):
    txt = gbdt_pmml(n_trees=5, depth=3, n_features=4, seed=1)
    txt = _decimal_thresholds(txt).replace("<MiningModel ", '<MiningModel x-mathContext="float" ', 1)
    c = CompiledPmml.from_string(txt)
    assert c.model.math_context == "float"
    seg = c.model.segments[0].model
    assert seg.math_context == "float"  # inherited by the segments
    vals = []
    stack = [seg.root]
    while stack:
        nd = stack.pop()
        if getattr(nd.predicate, "value", None) is not None:
            vals.append(float(nd.predicate.value))
        stack.extend(nd.children)
    assert vals and all(float(np.float32(v)) == v for v in vals)


def test_float_context_changes_edge_decisions(reader):
    base = _decimal_thresholds(gbdt_pmml(n_trees=40, depth=5, n_features=6, seed=2))
    c64 = CompiledPmml.from_string(base)
    c32 = CompiledPmml.from_string(_float_ctx(base))
    X = _edge_inputs(c32)
    s64, v64 = c64.score_matrix_oracle(X)
    s32, v32 = c32.score_matrix_oracle(X)
    assert (v64 == v32).all()
    assert (s64 != s32).mean() > 0.05  # the edge rows route differently
    # float32 segment sums: the float oracle equals an explicit float32 left-to-right sum (+ the
    # double Targets rescale of the base score)
    ev = c32.evaluator
    assert ev.method == "sum"
    cols = c32.columns(X.astype(np.float64))
    acc = np.zeros(len(X), dtype=np.float32)
    for sub in ev.sub:
        acc = acc + sub.evaluate(cols).value.astype(np.float32)
    t = ev.target
    want = acc.astype(np.float64) * (t.rescale_factor if t else 1.0) + (t.rescale_constant if t else 0.0)
    np.testing.assert_array_equal(s32, want)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["auto", "pointer"])
def test_float_context_gpu_matches_float_oracle(gpu, layout):
    """The fp32 kernels agree with the float-context oracle: identical decisions on the edge rows;
    sums differ only by fp32 re-association (documented tolerance: 1e-5 absolute, a few ulp of the
    partial sums, vs ~0.1 for one leaf routed differently)."""
    txt = _float_ctx(_decimal_thresholds(gbdt_pmml(n_trees=200, depth=6, n_features=12, seed=3)))
    c = CompiledPmml.from_string(txt)
    X = _edge_inputs(c, n=20000, seed=4)
    ref, vref = c.score_matrix_oracle(X)
    s, v = c.plan(gpu, layout=layout).score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    assert (v == vref).all()
    # fp32 re-association of the 200-leaf sum and the fp32 base-score add: a few ulp of the partial
    # sums (|partial| <= ~4 here, ulp 4.8e-7), i.e. far below one leaf (~0.1) of a different route
    err = np.abs(s[v] - ref[v])
    print(f"float-context max |gpu - oracle| = {err.max():.3g}")
    assert err.max() < 1e-5
    # ... while a double evaluation of the same document routes the edge rows differently
    ref64, _ = CompiledPmml.from_string(txt.replace(' x-mathContext="float"', "")).score_matrix_oracle(X)
    assert (np.abs(ref64[v] - ref[v]) > 1e-3).mean() > 0.05
