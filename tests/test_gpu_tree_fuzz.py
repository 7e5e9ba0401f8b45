"""Randomized tree ensembles on the GPU with the automatic plan choice (whatever layout, variant,
row tile and accumulation mode `TreePlan` picks for the shape) vs the float64 oracle: GBDT
regression / binary / multiclass chains and majority-vote random forests, depth 1-16, 1-300
trees, 1-300 features, both missing-value strategies, missing rates up to 30 %, batches from a
single row to 20k rows. Catches routing edge cases between the PERFECT, pointer and general
kernels that the hand-written cases do not pin."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

pytestmark = pytest.mark.gpu


def _shape(seed):
    rng = np.random.default_rng(7000 + seed)
    kind = ["regression", "binary", "multiclass", "rf"][int(rng.integers(0, 4))]
    depth = int(rng.integers(1, 17))
    n_trees = int(rng.integers(1, 301 if depth <= 10 else 61))
    F = int(rng.choice([1, 3, 8, 32, 90, 300]))
    missing = float(rng.choice([0.0, 0.02, 0.3]))
    strategy = str(rng.choice(["defaultChild", "nullPrediction"]))
    rows = int(rng.choice([1, 63, 257, 5000, 20_000]))
    p_split = float(rng.uniform(0.6, 0.95))
    return kind, depth, n_trees, F, missing, strategy, rows, p_split, int(rng.integers(0, 1 << 30))


@pytest.mark.parametrize("seed", gpu_seeds(32, 10))
def test_random_tree_ensembles_match_oracle(gpu, seed):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    kind, depth, n_trees, F, missing, strategy, rows, p_split, s = _shape(seed)
    if kind == "rf":
        txt = random_forest_pmml(n_trees=n_trees, depth=depth, n_features=F, n_classes=3, seed=s, p_split=p_split,
                                 missing_strategy=strategy)
    else:
        txt = gbdt_pmml(n_trees=n_trees, depth=depth, n_features=F, seed=s, objective=kind, p_split=p_split,
                        missing_strategy=strategy, n_classes=4)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)  # raises NotLowerable instead of falling back to the host
    X = stream_matrix(rows, F, seed=seed, missing_rate=missing)
    sc, v = plan.score(X)
    sc, v = sc.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    info = (kind, depth, n_trees, F, missing, strategy, rows, type(plan).__name__)
    assert (v == vref).all(), info
    if not v.any():  # e.g. nullPrediction with 30 % missing values: every row void, as in the oracle
        return
    if kind in ("rf", "multiclass"):  # labels: fp32 vote / softmax ties may differ in rare rows
        assert (sc[v] == ref[v]).mean() > 0.995, info
    else:
        np.testing.assert_allclose(sc[v], ref[v], rtol=1e-5, atol=1e-4, err_msg=str(info))
