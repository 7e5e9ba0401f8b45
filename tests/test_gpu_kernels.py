"""HIP kernel numerics vs the float64 host oracle (the semantic reference for every model type).

Tolerances: tree ensembles sum leaf values in fp32 (|err| ≲ 1e-5 for 1000 trees of ~0.1-scale
leaves); split decisions are exact for fp32 inputs (directionally rounded thresholds), so the
*selected leaves* — and therefore classification labels — must match exactly.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gpu_np(plan, X, **kw):
    s, v = plan.score(X, **kw)
    return s.cpu().numpy(), v.cpu().numpy()


def test_native_library_loaded(gpu):
    from flink_jpmml_amd.ops import _lib

    lib = _lib.load()
    assert lib._name.endswith("_pmml_kernels.so")


def test_kmeans_goldens_on_gpu(gpu, fixtures_dir):
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import ClusterPlan

    c = CompiledPmml.load(fixtures_dir["kmeans"])
    plan = c.plan(gpu)
    assert isinstance(plan, ClusterPlan)
    X = np.array([[1, 1, 1, 1], [1, 2, 3, 4], [1, np.nan, 2, np.nan], [np.nan] * 4, [6.9, 3.1, 5.8, 2.1]], float)
    s, v = _gpu_np(plan, X)
    assert s[:3].tolist() == [3.0, 4.0, 3.0]
    assert v.tolist() == [True, True, True, False, True]
    ref, vref = c.score_matrix_oracle(X)
    assert (vref == v).all() and np.allclose(ref[v], s[v])
    s0, v0 = _gpu_np(plan, X[2:3], replace_nan=0.0)
    assert v0[0] and s0[0] == 3.0


def test_kmeans_random_parity(gpu, fixtures_dir):
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.load(fixtures_dir["kmeans"])
    rng = np.random.default_rng(0)
    X = rng.uniform(0, 8, (100_000, 4))
    X[rng.random(X.shape) < 0.1] = np.nan
    s, v = _gpu_np(c.plan(gpu), X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.9999  # fp32 vs fp64 distance near-ties only


@pytest.mark.parametrize("depth,trees,feat,missing", [(6, 200, 32, 0.05), (3, 17, 5, 0.0), (8, 50, 64, 0.1),
                                                      (10, 8, 16, 0.02)])
def test_gbdt_regression_parity(gpu, depth, trees, feat, missing):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=trees, depth=depth, n_features=feat, seed=depth))
    plan = c.plan(gpu)
    assert plan.layout == "perfect"
    X = stream_matrix(20_000, feat, seed=1, missing_rate=missing)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert np.max(np.abs(s - ref)) < 2e-5 * max(1.0, trees / 100)


def test_gbdt_split_and_pointer_layouts(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=300, depth=7, n_features=24, seed=11))
    X = stream_matrix(3000, 24, seed=4, missing_rate=0.05)
    ref, vref = c.score_matrix_oracle(X)
    perfect = c.plan(gpu)
    for splits in (1, 4, 19):
        s, v = perfect.score(X) if splits == 1 else (None, None)
        if splits > 1:
            import torch

            Xt = torch.from_numpy(X.astype(np.float32)).to(gpu)
            so = torch.empty(len(X), device=gpu)
            vo = torch.empty(len(X), dtype=torch.uint8, device=gpu)
            perfect.launch(Xt, so, vo, splits=splits)
            s, v = so, vo.bool()
        s, v = s.cpu().numpy(), v.cpu().numpy()
        assert (v == vref).all()
        assert np.max(np.abs(s - ref)) < 1e-4
    for schedule, order in (("lockstep", "bfs"), ("lockstep", "dfs"), ("refill", "bfs")):
        pointer = c.plan(gpu, layout="pointer", pointer_schedule=schedule, node_order=order)
        assert pointer.layout == "pointer" and (pointer.variant == 16) == (schedule == "refill")
        s, v = _gpu_np(pointer, X)
        assert (v == vref).all() and np.max(np.abs(s - ref)) < 1e-4


def test_gbdt_binary_chain(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=120, depth=5, n_features=20, seed=5, objective="binary"))
    plan = c.plan(gpu)
    X = stream_matrix(50_000, 20, seed=3, missing_rate=0.03)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    # labels: only rows whose probability sits within fp32 noise of 0.5 may differ
    assert (s == ref).mean() > 0.9999


def test_random_forest_vote(gpu):
    from flink_jpmml_amd.bench.synth import random_forest_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(random_forest_pmml(n_trees=101, depth=7, n_features=16, n_classes=3, seed=2))
    X = stream_matrix(20_000, 16, seed=8, missing_rate=0.02)
    s, v = _gpu_np(c.plan(gpu), X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s == ref).all()  # integer vote counts are exact in fp32


def test_iris_logistic_regression(gpu):
    from flink_jpmml_amd.assets import IRIS_FIELDS  # noqa: F401
    from flink_jpmml_amd.bench.synth import iris_logistic_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import LinearPlan

    c = CompiledPmml.from_string(iris_logistic_pmml())
    plan = c.plan(gpu)
    assert isinstance(plan, LinearPlan)
    rng = np.random.default_rng(0)
    X = rng.uniform([4, 2, 1, 0], [8, 4.5, 7, 2.5], (10_000, 4))
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    # categories are non-numeric strings -> no numeric score, every row EmptyScore
    assert not v.any()


def test_interval_return_invalid_on_gpu(gpu, fixtures_dir):
    """kmeans40 with returnInvalid semantics vs asIs: rows outside the DataField interval."""
    from flink_jpmml_amd.assets import kmeans_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(kmeans_pmml("4.3", invalid_treatment="returnInvalid"))
    X = np.array([[1, 1, 1, 1], [5, 3, 2, 1], [7.9, 4.4, 6.9, 2.5], [4.3, 2.0, 1.0, 0.1]], float)
    s, v = _gpu_np(c.plan(gpu), X)
    ref, vref = c.score_matrix_oracle(X)
    assert v.tolist() == vref.tolist() == [False, True, True, True]
    assert np.allclose(s[v], ref[v])


def test_streaming_scorer_pipeline_matches_plan(gpu):
    import torch

    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.engine import StreamingScorer

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=100, depth=6, n_features=16, seed=9))
    plan = c.plan(gpu)
    X = stream_matrix(50_001, 16, seed=3, missing_rate=0.01)
    ref_s, ref_v = plan.score(X)
    for direct in (True, False):
        scorer = StreamingScorer(plan, micro_batch=4096, depth=3, max_rows=50_001, direct_host_output=direct)
        assert scorer.direct == direct
        Xp = torch.from_numpy(X).pin_memory()
        sh = torch.full((len(X),), -7.0).pin_memory()
        vh = torch.zeros(len(X), dtype=torch.uint8).pin_memory()
        for _ in range(3):  # several steps reuse the ring + output buffers
            h = scorer.submit(Xp, sh, vh)
        scorer.wait(h)
        # micro-batches of 4096 rows use the tree-split kernel (different fp32 summation order)
        assert torch.equal(vh.bool(), ref_v.cpu())
        assert torch.allclose(sh, ref_s.cpu(), atol=1e-5, rtol=0)
        assert torch.equal(h.score_dev.cpu(), sh)  # device mirror == zero-copy host sink


def test_stream_dsl_on_gpu(gpu, fixtures_dir):
    from flink_jpmml_amd import DenseVector, ModelReader, SparseVector
    from flink_jpmml_amd.domain import EmptyScore, Prediction, Score
    from flink_jpmml_amd.stream import StreamExecutionEnvironment

    vecs = [DenseVector(1, 1, 1, 1), SparseVector(4, [0, 1, 2, 3], [1, 2, 3, 4]), SparseVector(4, [0, 2], [1, 2]),
            DenseVector(1, 2, 3)] * 50
    env = StreamExecutionEnvironment()
    out = env.from_collection(vecs).quick_evaluate(ModelReader(fixtures_dir["kmeans"]), batch_size=64,
                                                   device=gpu).collect()
    exp = [Prediction(Score(3.0)), Prediction(Score(4.0)), Prediction(Score(3.0)), Prediction(EmptyScore)] * 50
    assert [p for p, _ in out] == exp


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 5e-2)])
def test_mlp_regression_mfma(gpu, precision, tol):
    """3-layer NeuralNetwork on the fused MFMA kernel: fp32 MFMA (exact FMA chain) matches the
    fp64 oracle to ~1e-5 relative; bf16 MFMA (bf16 operands, fp32 accumulate) to a few 1e-3."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.nn_plans import MlpPlan

    c = CompiledPmml.from_string(mlp_pmml(n_features=40, hidden=(96, 70), n_out=1, seed=4))
    plan = c.plan(gpu, precision=precision)
    assert isinstance(plan, MlpPlan)
    X = stream_matrix(10_000, 40, seed=2)
    X[5, 3] = np.nan  # a missing input invalidates the row (PMML NN rule)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and not v[5]
    scale = np.max(np.abs(ref[vref]))
    assert np.max(np.abs(s[v] - ref[v])) < tol * max(1.0, scale)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_mlp_classification_softmax(gpu, precision):
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(mlp_pmml(n_features=16, hidden=(64,), n_out=5, seed=1, activation="tanh",
                                          classification=True))
    X = stream_matrix(20_000, 16, seed=6)
    s, v = _gpu_np(c.plan(gpu, precision=precision), X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    agree = (s == ref).mean()
    assert agree > (0.9999 if precision == "fp32" else 0.98)


@pytest.mark.parametrize("kernel", ["radialBasis", "linear", "polynomial", "sigmoid"])
def test_svm_kernels(gpu, kernel):
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.nn_plans import SvmPlan

    c = CompiledPmml.from_string(svm_pmml(n_features=12, n_sv=100, seed=3, kernel=kernel))
    plan = c.plan(gpu)
    assert isinstance(plan, SvmPlan)
    X = stream_matrix(20_000, 12, seed=4)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert not v.any() or (s[v] == ref[v]).mean() > 0.999


def test_svm_regression(gpu):
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(svm_pmml(n_features=10, n_sv=64, seed=5, classification=False))
    X = stream_matrix(5000, 10, seed=1)
    s, v = _gpu_np(c.plan(gpu), X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and np.max(np.abs(s - ref)) < 1e-4


def test_plan_state_roundtrip(gpu):
    """What broadcast_plan ships over RCCL: export_state -> from_state scores identically."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import DevicePlan

    for txt, F in ((gbdt_pmml(n_trees=50, depth=5, n_features=12, seed=2), 12), (mlp_pmml(n_features=12), 12)):
        c = CompiledPmml.from_string(txt)
        p = c.plan(gpu)
        meta, tensors = p.export_state()
        q = DevicePlan.from_state(meta, {k: v.clone() for k, v in tensors.items()}, gpu)
        X = stream_matrix(3000, F, seed=5)
        s1, v1 = p.score(X)
        s2, v2 = q.score(X)
        assert (s1 == s2).all() and (v1 == v2).all()


# ------------------------------------------------------------------ derived fields (derive.hip)


def test_derived_regression_program_on_gpu(gpu):
    """Every DerivedField kind through the derive kernel, then the linear kernel (mask fixup)."""
    from test_derive import inputs, regression_doc

    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.derive import DerivedPlan, emulate

    c = CompiledPmml.from_string(regression_doc())
    plan = c.plan(gpu)
    assert isinstance(plan, DerivedPlan)
    X = inputs(20_000, seed=7)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=2e-5, atol=2e-5)
    # the device program equals its numpy twin column for column
    import torch

    P, _ = c.prepare(X)
    Xt = torch.from_numpy(X.astype(np.float32)).to(gpu)
    Xa, ok = plan._buffers(None, len(X))
    sc, va = plan.alloc_outputs(len(X))
    plan.launch(Xt, sc, va)
    torch.cuda.synchronize()
    np.testing.assert_allclose(Xa.cpu().numpy(), emulate(plan.program, P), rtol=1e-6, atol=1e-7, equal_nan=True)


def test_derived_tree_program_on_gpu(gpu):
    from test_derive import inputs, tree_doc

    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.derive import DerivedPlan
    from flink_jpmml_amd.runtime.plans import DevicePlan, TreePlan

    c = CompiledPmml.from_string(tree_doc())
    plan = c.plan(gpu)
    assert isinstance(plan, DerivedPlan) and isinstance(plan.inner, TreePlan)
    X = inputs(30_000, seed=2)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and (s[v] == ref[v]).all()
    meta, tensors = plan.export_state()  # RCCL replication of a derived plan
    q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, gpu)
    s2, v2 = _gpu_np(q, X)
    assert (s2 == s).all() and (v2 == v).all()


def test_float_cast_gbdt_aliases_on_gpu(gpu):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=100, depth=6, n_features=16, seed=9, float_casts=True))
    plan = c.plan(gpu)
    assert isinstance(plan, TreePlan)  # casts alias their input columns: no derive pass
    X = stream_matrix(20_000, 16, seed=3, missing_rate=0.03)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and np.max(np.abs(s - ref)) < 2e-5


# ------------------------------------------------------------------ null-on-missing trees, fp8 leaves


@pytest.mark.parametrize("kind,layout", [("regression", "perfect"), ("regression", "pointer"), ("rf", "perfect"),
                                         ("rf", "pointer"), ("regression", "refill"), ("rf", "refill")])
def test_null_prediction_trees_on_gpu(gpu, kind, layout):
    from flink_jpmml_amd.bench.synth import gbdt_pmml, random_forest_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    if kind == "rf":
        txt = random_forest_pmml(n_trees=40, depth=6, n_features=10, n_classes=3, seed=4,
                                 missing_strategy="nullPrediction")
    else:
        txt = gbdt_pmml(n_trees=80, depth=5, n_features=10, seed=3, missing_strategy="nullPrediction")
    c = CompiledPmml.from_string(txt)
    X = stream_matrix(20_000, 10, seed=6, missing_rate=0.01)
    ref, vref = c.score_matrix_oracle(X)
    assert 0 < vref.sum() < len(X)
    opts = dict(layout="pointer", pointer_schedule="refill") if layout == "refill" else dict(layout=layout)
    s, v = _gpu_np(c.plan(gpu, **opts), X)
    assert (v == vref).all()
    if kind == "rf":
        assert (s[v] == ref[v]).all()
    else:
        assert np.max(np.abs(s[v] - ref[v])) < 2e-5


def test_fp8_leaf_chain_on_gpu(gpu):
    """BASELINE config 5: GBDT chain + logistic calibrator with e4m3 leaves. Decisions are exact;
    the tolerance is the leaf quantisation (3 mantissa bits, one global scale)."""
    from test_lowering import emulate_leaf8

    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=300, depth=6, n_features=24, seed=8, objective="binary"))
    p8 = c.plan(gpu, precision="fp8")
    assert p8.variant & 3 == 2 and p8.rec_words < c.plan(gpu).rec_words
    X = stream_matrix(30_000, 24, seed=1)
    probs = torch_probs = None
    import torch

    Xt = torch.from_numpy(X).to(gpu)
    s8, v8 = p8.alloc_outputs(len(X))
    probs = torch.empty((len(X), 2), device=gpu)
    p8.launch(Xt, s8, v8, probs=probs)
    torch.cuda.synchronize()
    spec, acc8, _ = emulate_leaf8(c, X)
    e = spec.epi
    p_emul = 1.0 / (1.0 + np.exp(-(e["a"] * acc8.astype(np.float64) + e["b"])))
    torch_probs = probs[:, 0].cpu().numpy()
    assert np.max(np.abs(torch_probs - p_emul)) < 1e-4  # kernel == fp8 emulation (fp32 sum order)
    ref, vref = c.score_matrix_oracle(X)
    assert v8.bool().all().item() and vref.all()
    assert (s8.cpu().numpy() == ref).mean() > 0.97  # labels vs the fp64 oracle on fp32 leaves


@pytest.mark.parametrize("precision,feat", [("fp32", 32), ("fp32", 48), ("fp8", 24), ("fp8", 40)])
def test_nan_planes_match_per_node_missing_path(gpu, precision, feat):
    """Tiles with missing values: the NaN-plane fast traversal == the per-node missing test
    (bit-identical scores: same trees, same summation order)."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import VAR_NAN_FAST, VAR_NAN_PLANES

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=120, depth=6, n_features=feat, seed=feat))
    fast = c.plan(gpu, precision=precision)
    slow = c.plan(gpu, precision=precision, nan_mode="off")
    if precision == "fp8" and feat > 32:  # 16-bit feature offsets of the fp8 metas: no second plane
        assert not fast.variant & (VAR_NAN_FAST | VAR_NAN_PLANES)
    else:
        assert fast.variant & VAR_NAN_FAST and not slow.variant & VAR_NAN_FAST
    X = stream_matrix(40_000, feat, seed=2, missing_rate=0.03)
    s1, v1 = _gpu_np(fast, X)
    s0, v0 = _gpu_np(slow, X)
    assert (v1 == v0).all() and np.array_equal(s1[v1], s0[v0])
    if precision == "fp32":
        ref, vref = c.score_matrix_oracle(X)
        assert (v1 == vref).all() and np.max(np.abs(s1 - ref)) < 2e-5 * 1.2


@pytest.mark.parametrize("strategy", ["defaultChild", "nullPrediction"])
def test_categorical_splits_on_gpu(gpu, strategy):
    """isIn / isNotIn / == / != splits: derive-kernel membership columns + the tree kernel."""
    from test_derive import cat_inputs, categorical_tree_doc

    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.derive import DerivedPlan

    c = CompiledPmml.from_string(categorical_tree_doc(strategy))
    plan = c.plan(gpu)
    assert isinstance(plan, DerivedPlan)
    X = cat_inputs(20_000, seed=3)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and (s[v] == ref[v]).all()


@pytest.mark.parametrize("strategy,no_true", [("none", "returnNullPrediction"), ("lastPrediction", "returnLastPrediction"),
                                              ("nullPrediction", "returnNullPrediction"),
                                              ("defaultChild", "returnLastPrediction")])
def test_general_tree_layout_on_gpu(gpu, strategy, no_true):
    """Multiway / compound / set predicates through the predicate-VM kernel vs the fp64 oracle."""
    from test_general_tree import general_inputs, general_tree_doc

    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    for seed in range(2):
        c = CompiledPmml.from_string(general_tree_doc(seed, strategy, no_true))
        plan = c.plan(gpu)
        assert getattr(plan, "inner", plan).layout == "general"  # set splits may add a derive pass
        X = general_inputs(20_000, seed)
        s, v = _gpu_np(plan, X)
        ref, vref = c.score_matrix_oracle(X)
        assert (v == vref).all()
        np.testing.assert_allclose(s[v], ref[v], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("classification", [False, True])
def test_general_tree_ensemble_on_gpu(gpu, classification):
    from test_general_tree import general_inputs, general_tree_doc

    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.plans import DevicePlan

    c = CompiledPmml.from_string(general_tree_doc(5, "defaultChild", "returnLastPrediction", n_trees=25,
                                                  classification=classification))
    plan = c.plan(gpu)
    X = general_inputs(20_000, 9)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-5, atol=1e-5)
    meta, tensors = plan.export_state()
    q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, gpu)
    s2, v2 = _gpu_np(q, X)
    assert (s2 == s).all() and (v2 == v).all()
