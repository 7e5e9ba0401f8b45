"""Wide PERFECT tree kernel on the GPU: multi-class accumulation modes (K-class GBDT chains in
class slots, weighted / packed-u8 majority votes) and wide records (row tiles of 128 / 64 rows,
staged-column compaction) vs the float64 oracle. CPU twins of every case: tests/test_wide_modes.py
(numpy emulation of the same packed tensors)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(gpu, txt, n, F, missing, seed=1, **kw):
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **kw)
    X = stream_matrix(n, F, seed=seed, missing_rate=missing)
    s, v = plan.score(X)
    ref, vref = c.score_matrix_oracle(X)
    return plan, s.cpu().numpy(), v.cpu().numpy(), ref, vref


@pytest.mark.parametrize("K", [3, 5, 8])
def test_multiclass_chain_slot_mode_on_gpu(gpu, K):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    plan, s, v, ref, vref = _run(gpu, gbdt_pmml(n_trees=60, depth=6, n_features=20, objective="multiclass",
                                                n_classes=K, seed=K), 40_000, 20, 0.03, seed=K)
    assert plan.variant & 3 == 1 and plan.mode == 1
    assert (v == vref).all()
    assert (s == ref).mean() > 0.9999  # softmax near-ties in fp32 only


def test_multiclass_chain_twelve_classes_general_slots_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    plan, s, v, ref, vref = _run(gpu, gbdt_pmml(n_trees=10, depth=4, n_features=12, objective="multiclass",
                                                n_classes=12, seed=2), 20_000, 12, 0.02)
    assert plan.mode == 0 and plan.C == 12
    assert (v == vref).all() and (s == ref).mean() > 0.9999


def test_forest_vote8_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import random_forest_pmml

    plan, s, v, ref, vref = _run(gpu, random_forest_pmml(n_trees=500, depth=8, n_features=32, n_classes=3, seed=4),
                                 30_000, 32, 0.02)
    assert plan.mode == 3 and plan.variant & 3 == 2  # class codes in the last-level metas
    assert (v == vref).all() and (s == ref).all()


def test_forest_class_mode_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import random_forest_pmml

    plan, s, v, ref, vref = _run(gpu, random_forest_pmml(n_trees=64, depth=6, n_features=16, n_classes=7, seed=5),
                                 30_000, 16, 0.02)
    assert plan.mode == 2
    assert (v == vref).all() and (s == ref).all()


def test_null_prediction_forest_wide_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import random_forest_pmml

    plan, s, v, ref, vref = _run(gpu, random_forest_pmml(n_trees=30, depth=5, n_features=10, n_classes=3, seed=6,
                                                         missing_strategy="nullPrediction"), 20_000, 10, 0.01)
    assert plan.variant & 3 in (1, 2) and 0 < vref.sum() < len(vref)
    assert (v == vref).all() and (s[v] == ref[v]).all()


@pytest.mark.parametrize("F,precision", [(100, "fp32"), (200, "fp32"), (100, "fp8")])
def test_wide_records_on_gpu(gpu, F, precision):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    plan, s, v, ref, vref = _run(gpu, gbdt_pmml(n_trees=200, depth=6, n_features=F, seed=F), 20_000, F, 0.02,
                                 precision=precision)
    assert plan.variant & 3 == (2 if precision == "fp8" else 1) and plan.rows_wide in (128, 64)
    assert (v == vref).all()
    tol = 2e-4 if precision == "fp32" else 200 * 0.1 * 4 / 16  # e4m3 leaves: |rel err| <= 1/16
    assert np.max(np.abs(s - ref)) < tol


def test_feature_compaction_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    plan, s, v, ref, vref = _run(gpu, gbdt_pmml(n_trees=4, depth=3, n_features=400, seed=9), 10_000, 400, 0.05)
    assert plan.feat_map is not None and plan.rows_wide == 256
    assert (v == vref).all() and np.max(np.abs(s - ref)) < 1e-5


def test_folded_derived_fields_on_gpu(gpu):
    """Monotone derived fields (StandardScaler / NormContinuous / decreasing affine) folded into the
    split thresholds: the tree kernel reads the raw inputs (no derive pass) and matches the oracle."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    plan, s, v, ref, vref = _run(gpu, gbdt_pmml(n_trees=200, depth=6, n_features=32, scaled=True, seed=7),
                                 60_000, 32, 0.03, seed=8)
    assert type(plan).__name__ == "TreePlan" and plan.variant & 3 == 1
    assert (v.astype(bool) == vref).all()
    assert np.max(np.abs(s[vref] - ref[vref])) < 1e-4
