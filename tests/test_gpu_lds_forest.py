"""GPU twin of test_lds_layout.py: the LDS-resident deep-forest walk (``tree_lds.hip``) against
the float64 oracle and the pointer walk."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,missing", [("gbdt", "defaultChild"), ("gbdt", "nullPrediction"),
                                          ("rf", "defaultChild")])
def test_lds_forest_matches_oracle_and_pointer(gpu, kind, missing):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import VAR_POINTER_LDS

    gen = gbdt_pmml if kind == "gbdt" else random_forest_pmml
    txt = gen(n_trees=48, depth=13, n_features=32, seed=7, p_split=0.85)
    if missing == "nullPrediction":
        txt = txt.replace('missingValueStrategy="defaultChild"', 'missingValueStrategy="nullPrediction"')
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, layout="pointer", node_format="lds")
    assert plan.variant == VAR_POINTER_LDS
    X = stream_matrix(70_001, 32, seed=3, missing_rate=0.02)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and v.any()
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=2e-5 if kind == "gbdt" else 0)
    ps, pv = c.plan(gpu, layout="pointer").score(X)
    ps, pv = ps.cpu().numpy(), pv.cpu().numpy().astype(bool)
    assert (pv == v).all()
    np.testing.assert_allclose(ps[v], s[v], rtol=0, atol=2e-5 if kind == "gbdt" else 0)


def test_lds_forest_small_batches(gpu):
    """Row counts below one tile and not a tile multiple; one-slice forests."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=5, depth=11, n_features=12, seed=2, p_split=0.8))
    plan = c.plan(gpu, layout="pointer", node_format="lds")
    for n in (1, 37, 513, 4097):
        X = stream_matrix(n, 12, seed=n, missing_rate=0.05)
        s, v = plan.score(X)
        ref, vref = c.score_matrix_oracle(X)
        v = v.cpu().numpy().astype(bool)
        assert (v == vref).all()
        np.testing.assert_allclose(s.cpu().numpy()[v], ref[v], rtol=0, atol=2e-5)
