"""Wide NeuralNetworks on the fused MFMA GEMM (``ops/csrc/gemm.hip``, ``WideMlpPlan``).

CPU: the plan's packed operands (unit-major bf16 weights padded to the kernel tiles, fp32 biases,
the input stage) run through a numpy model of the kernels' arithmetic — bf16 operands, fp32
accumulation, bf16 activations between layers — and must reproduce the float64 oracle within bf16
tolerance. The fp32 variant (default fp32 policy: exact-fp32 MFMA, fp32 activations) must match
the oracle to fp32 rounding. GPU: the kernels against the same model (tight) and the oracle."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml

SHAPES = [
    dict(n_features=32, hidden=(1024,), n_out=1, activation="rectifier"),
    dict(n_features=600, hidden=(300,), n_out=40, activation="tanh", classification=True),
    dict(n_features=40, hidden=(300, 1024), n_out=1, activation="logistic"),
    dict(n_features=21, hidden=(512,), n_out=5, activation="tanh", classification=True),
    dict(n_features=16, hidden=(64,) * 9, n_out=1, activation="rectifier"),
]
_ACT = {0: lambda z: z, 1: lambda z: 1 / (1 + np.exp(-z)), 2: np.tanh, 3: lambda z: np.maximum(z, 0)}


def _bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16).float().numpy()


def emulate_wide(plan, X):
    """numpy model of nn_prep_kernel + gemm_kernel (hidden + output layer decode)."""
    X = np.asarray(X, np.float32)
    idx = plan.in_index.cpu().numpy()
    x = X[:, idx]
    sc, sh, ms = (t.cpu().numpy() for t in (plan.in_scale, plan.in_shift, plan.in_missing))
    z = np.where(np.isnan(x), ms, x * sc + sh)
    ok = ~np.isnan(z).any(axis=1)
    H = np.zeros((len(X), plan.k0), np.float32)
    H[:, : plan.n_in] = np.nan_to_num(z)
    rnd = _bf16 if plan.bf16 else (lambda a: np.asarray(a, np.float32))
    H = rnd(H)
    W = plan.wts.float().cpu().numpy()
    B = plan.bss.cpu().numpy()
    for li, (kp, mp, act, thr, wo, bo) in enumerate(plan.dims):
        Wt = W[wo: wo + mp * kp].reshape(mp, kp)
        Z = (H[:, :kp].astype(np.float64) @ Wt.T.astype(np.float64)).astype(np.float32) + B[bo: bo + mp]
        Z = _ACT[act](Z).astype(np.float32)
        H = rnd(Z) if li < len(plan.dims) - 1 else Z
    out = H[:, : plan.n_out]
    if plan.is_classification:
        P = np.exp(out - out.max(1, keepdims=True)) if plan.final_norm == 1 else out
        if plan.final_norm:
            P = P / P.sum(1, keepdims=True)
        lab = P.argmax(1)
        s = plan.table.cpu().numpy()[lab].astype(np.float64)
    else:
        s = plan.out_a * out[:, 0].astype(np.float64) + plan.out_b
    return np.where(ok, s, np.nan), ok


@pytest.mark.parametrize("shape", SHAPES, ids=lambda d: "x".join(map(str, d["hidden"])))
def test_wide_plan_packing_matches_oracle(shape):
    from flink_jpmml_amd.runtime.nn_plans import WideMlpPlan
    from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(mlp_pmml(seed=5, **shape))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"), precision="bf16")
    assert isinstance(plan, WideMlpPlan)
    assert all(kp % 64 == 0 and mp % (32 if i == len(plan.dims) - 1 else 256) == 0
               for i, (kp, mp, *_) in enumerate(plan.dims))
    X = stream_matrix(3000, shape["n_features"], seed=2, missing_rate=0.01)
    s, v = emulate_wide(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if shape.get("classification"):
        assert (s[v] == ref[v]).mean() > 0.98
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        assert np.abs(s[v] - ref[v]).max() < 3e-2 * scale


@pytest.mark.parametrize("shape", SHAPES, ids=lambda d: "x".join(map(str, d["hidden"])))
def test_fp32_policy_runs_fp32_wide_gemm(shape):
    """fp32 precision policy: wide layers stay fp32 — on the fused GEMM's exact-fp32 MFMA variant
    (not a library GEMM); bf16 operands are opt-in. Packed fp32 operands reproduce the oracle."""
    from flink_jpmml_amd.runtime.nn_plans import WideMlpPlan
    from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(mlp_pmml(seed=5, **shape))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, WideMlpPlan) and plan.bf16 == 0 and plan.wts.dtype == torch.float32
    X = stream_matrix(2000, shape["n_features"], seed=2, missing_rate=0.01)
    s, v = emulate_wide(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if shape.get("classification"):
        assert (s[v] == ref[v]).mean() > 0.999
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        assert np.abs(s[v] - ref[v]).max() < 1e-4 * scale


def test_wide_plan_covers_many_outputs_and_inputs():
    """More than 32 output neurons (32-unit output groups + the streaming wide decode) and more
    than 512 inputs (the input stage spreads a row's chunks over a wave) stay on the hand-written
    GEMM; only past 1024 outputs do library GEMMs take over."""
    from flink_jpmml_amd.runtime.nn_plans import GemmMlpPlan, WideMlpPlan
    from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(mlp_pmml(n_features=8, hidden=(300,), n_out=40, classification=True, seed=1))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, WideMlpPlan) and plan.dims[-1][1] == 64 and not plan._fused_head()
    c = CompiledPmml.from_string(mlp_pmml(n_features=700, hidden=(300,), n_out=1, seed=1))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, WideMlpPlan) and plan.k0 == 704
    c = CompiledPmml.from_string(mlp_pmml(n_features=4, hidden=(8,), n_out=1030, classification=True, seed=1))
    with lowering_dry_run():
        assert isinstance(compile_plan(c, torch.device("cpu")), GemmMlpPlan)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda d: "x".join(map(str, d["hidden"])))
def test_wide_gemm_kernels_on_gpu(gpu, shape, precision):
    from flink_jpmml_amd.runtime.nn_plans import WideMlpPlan

    c = CompiledPmml.from_string(mlp_pmml(seed=5, **shape))
    plan = c.plan(gpu, precision=precision)
    assert isinstance(plan, WideMlpPlan) and plan.bf16 == (precision == "bf16")
    X = stream_matrix(10_001, shape["n_features"], seed=3, missing_rate=0.01)  # not a multiple of 256
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy()
    es, ev = emulate_wide(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == ev).all() and (v == vref).all()
    fp32 = precision == "fp32"
    if shape.get("classification"):
        assert (s[v] == es[v]).mean() > 0.995
        assert (s[v] == ref[v]).mean() > (0.999 if fp32 else 0.98)
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        assert np.abs(s[v] - es[v]).max() < (1e-4 if fp32 else 5e-3) * scale  # same operands: summation order
        assert np.abs(s[v] - ref[v]).max() < (1e-4 if fp32 else 3e-2) * scale


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=100, hidden=(300,)), dict(n_features=150, hidden=(260, 300)),
                                   dict(n_features=40, hidden=(1024, 512))],
                         ids=["k128", "k192", "k1024"])
def test_phase_interleaved_gemm_matches_two_buffer_loop(gpu, shape):
    """The phase-interleaved bf16 hidden-layer kernels — the persistent gemm8p_kernel (default for
    K >= 128) and the one-tile gemm8_kernel (bit 12, K >= 512, or forced by bit 7): half-tile
    staging, counted vmcnt across raw barriers, staggered wave groups — must give the same bits as
    the 2-buffer loop (bit 12 at K < 512) on every hidden layer, including K = 128 / 192 (2 / 3
    slices, the pipeline's edge cases): the same MFMAs in the same k order."""
    c = CompiledPmml.from_string(mlp_pmml(seed=9, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_head = False  # every hidden layer through pmml_gemm_launch
    X = stream_matrix(5000, shape["n_features"], seed=4, missing_rate=0.01)
    s0, v0 = plan.score(X)
    for flags in (0x1000, 0x1080):  # one tile per workgroup: 2-buffer loop below K = 512 / gemm8_kernel forced
        plan.gemm_flags = flags
        try:
            s1, v1 = plan.score(X)
        finally:
            plan.gemm_flags = 0
        assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()]), hex(flags)
    ref, vref = c.score_matrix_oracle(X)
    s1, v1 = s1.cpu().numpy(), v1.cpu().numpy().astype(bool)
    assert (v1 == vref).all()
    assert np.abs(s1[v1] - ref[v1]).max() < 3e-2 * max(1.0, float(np.abs(ref[v1]).max()))


def test_fused_head_permutation_matches_accumulator_layout():
    """gemm8_kernel<true> feeds the last hidden layer's accumulators (a row per lane, units in the
    16 registers: unit (r & 3) + 8 (r >> 2) + 4 h for lane half h) straight into the output-layer
    MFMA as B fragments (k-step s = registers 8 s .. 8 s + 7, MFMA k = 8 h + e). The host-permuted
    weights must put, at the A-fragment position a lane reads (16 s + 8 h + e), the weight of the
    very unit that register carries."""
    from flink_jpmml_amd.runtime.nn_plans import fused_head_perm

    K = 1024
    perm = fused_head_perm(K)
    assert sorted(perm.tolist()) == list(range(K))  # a permutation inside every 32-unit group
    assert (perm // 32 == np.arange(K) // 32).all()
    for g in range(0, K, 32):
        for h in (0, 1):
            for s in (0, 1):
                for e in range(8):
                    r = 8 * s + e
                    unit = g + (r & 3) + 8 * (r >> 2) + 4 * h  # what accumulator register r carries
                    assert perm[g + 16 * s + 8 * h + e] == unit


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=32, hidden=(1024, 1024), n_out=1, activation="rectifier"),
                                   dict(n_features=21, hidden=(512,), n_out=5, activation="tanh",
                                        classification=True),
                                   dict(n_features=40, hidden=(300, 1024), n_out=3, activation="logistic",
                                        classification=True)],
                         ids=["reg1024x2", "cls512", "cls300x1024"])
def test_fused_output_layer_matches_separate_launch(gpu, shape):
    """The last hidden layer + output layer as one GEMM (the hidden activations never stored) give
    the unfused result up to fp32 summation order, and the oracle within bf16 tolerance."""
    c = CompiledPmml.from_string(mlp_pmml(seed=11, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    assert plan._fused_head()
    X = stream_matrix(20_001, shape["n_features"], seed=5, missing_rate=0.01)
    s1, v1 = plan.score(X)
    plan.fuse_head = False
    try:
        s0, v0 = plan.score(X)
    finally:
        plan.fuse_head = True
    assert torch.equal(v0, v1)
    s0, s1, v = s0.cpu().numpy(), s1.cpu().numpy(), v1.cpu().numpy().astype(bool)
    n = 4000  # the oracle walks connections in Python: its rows are a prefix
    ref, vref = c.score_matrix_oracle(X[:n])
    assert (v[:n] == vref).all()
    vo = v[:n]
    if shape.get("classification"):
        assert (s0[v] == s1[v]).mean() > 0.999
        assert (s1[:n][vo] == ref[vo]).mean() > 0.98
    else:
        scale = max(1.0, float(np.abs(ref[vo]).max()))
        assert np.abs(s1[v] - s0[v]).max() < 1e-4 * scale
        assert np.abs(s1[:n][vo] - ref[vo]).max() < 3e-2 * scale


@pytest.mark.gpu
def test_k64_first_layer_kernel_matches_256_tile(gpu):
    """The 128 x 256 / 4-wave first-layer kernel (gemm_k64_kernel, 3 workgroups per CU) runs the
    same MFMAs in the same k order as the 256 x 256 tile: identical bits (flag bit 6 forces the
    latter)."""
    c = CompiledPmml.from_string(mlp_pmml(n_features=32, hidden=(1024, 512), seed=13))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    assert plan.dims[0][0] == 64
    X = stream_matrix(9000, 32, seed=6, missing_rate=0.01)
    s0, v0 = plan.score(X)
    plan.gemm_flags = 0x40
    try:
        s1, v1 = plan.score(X)
    finally:
        plan.gemm_flags = 0
    assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=32, hidden=(1024, 1024, 1024)),
                                   dict(n_features=60, hidden=(512, 256), n_out=4, classification=True),
                                   dict(n_features=20, hidden=(300, 1024))],
                         ids=["1024x3", "cls512x256", "300x1024"])
def test_fused_input_stage_matches_separate_prep(gpu, shape):
    """Input stage fused into the first layer's GEMM (gemm_k64_kernel<true>: gather, NormContinuous,
    missing values, bf16 A tile built in LDS, row validity) gives the separate prep + GEMM bits."""
    c = CompiledPmml.from_string(mlp_pmml(seed=17, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_input = True  # opt-in (measured slower than the separate input stage)
    assert plan._fused_input(plan._fused_head())
    X = stream_matrix(12_345, shape["n_features"], seed=9, missing_rate=0.03)
    s1, v1 = plan.score(X)
    plan.fuse_input = False
    s0, v0 = plan.score(X)
    assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()])
    assert plan.in_contig == 1  # identity input map: the input stage's 16-byte gather
    plan.in_contig = 0
    try:
        s2, v2 = plan.score(X)  # the per-input gather
    finally:
        plan.in_contig = 1
    assert torch.equal(v0, v2) and torch.equal(s0[v0.bool()], s2[v2.bool()])
    ref, vref = c.score_matrix_oracle(X[:3000])  # the oracle walks connections in Python
    assert (v1[:3000].cpu().numpy().astype(bool) == vref).all()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=32, hidden=(1024, 1024, 512)), dict(n_features=40, hidden=(300, 260))],
                         ids=["1024x1024x512", "300x260"])
def test_wave_lds_epilogue_matches_direct_stores(gpu, shape):
    """Hidden-layer tiles leaving through the wave-private LDS scratch (16-byte stores, flag bit 5)
    equal the direct two-unit stores bit for bit."""
    c = CompiledPmml.from_string(mlp_pmml(seed=19, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_head = False  # every hidden layer stores its activations
    X = stream_matrix(7000, shape["n_features"], seed=2, missing_rate=0.01)
    s0, v0 = plan.score(X)
    plan.gemm_flags = 0x20
    try:
        s1, v1 = plan.score(X)
    finally:
        plan.gemm_flags = 0
    assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=32, hidden=(1024, 1024, 512)),
                                   dict(n_features=40, hidden=(300, 260), activation="tanh"),
                                   dict(n_features=24, hidden=(512, 768), activation="logistic", n_out=3,
                                        classification=True),
                                   dict(n_features=100, hidden=(512, 300))],
                         ids=["1024x1024x512", "300x260-tanh", "512x768-logistic", "k128-512x300"])
def test_transposed_accumulator_stores_match_direct_stores(gpu, shape):
    """The default bf16 hidden-layer epilogue (operands swapped so the accumulator tile is
    [unit][row]; v_permlane32_swap pairs the lane halves' unit runs into two 16-byte stores per lane,
    store_hidden_t) equals the direct two-unit stores of the [row][unit] tile (flag bit 8) bit for
    bit, on the K = 64 first-layer kernel, the two-buffer kernel (K = 128) and the phase-interleaved
    kernel, with and without the fused input stage; 41000 rows = 322 row tiles of the persistent K = 64 kernel (several per
    workgroup, a ragged last one)."""
    c = CompiledPmml.from_string(mlp_pmml(seed=23, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_head = False  # every hidden layer stores its activations
    X = stream_matrix(41_000, shape["n_features"], seed=4, missing_rate=0.01)
    s0, v0 = plan.score(X)
    plan.gemm_flags = 0x100
    try:
        s1, v1 = plan.score(X)
    finally:
        plan.gemm_flags = 0
    assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()])
    plan.gemm_flags = 0x200  # K = 64 layer: one tile per workgroup instead of the persistent kernel
    try:
        s3, v3 = plan.score(X)
    finally:
        plan.gemm_flags = 0
    assert torch.equal(v0, v3) and torch.equal(s0[v0.bool()], s3[v3.bool()])
    plan.fuse_input = True
    try:
        s2, v2 = plan.score(X)
    finally:
        plan.fuse_input = False
    assert torch.equal(v0, v2) and torch.equal(s0[v0.bool()], s2[v2.bool()])
    ref, vref = c.score_matrix_oracle(X[:3000])  # the oracle walks connections in Python
    assert (v0[:3000].cpu().numpy().astype(bool) == vref).all()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(n_features=32, hidden=(1024, 1024, 512)),
                                   dict(n_features=40, hidden=(300, 260), activation="tanh"),
                                   dict(n_features=24, hidden=(512, 768), activation="logistic", n_out=3,
                                        classification=True),
                                   dict(n_features=32, hidden=(1024, 1024, 1024, 512))],
                         ids=["1024x1024x512", "300x260-tanh", "512x768-logistic", "1024x3-512"])
def test_row_segment_stores_match_transposed_stores(gpu, shape):
    """The default 128-byte row-segment stores through a wave LDS scratch (store_hidden_seg) on the
    K = 64 persistent layer and on the phase-interleaved hidden kernel equal the store_hidden_t
    bits (flag bits 10 / 11); 41000 rows = a ragged last row tile."""
    c = CompiledPmml.from_string(mlp_pmml(seed=29, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_head = False
    X = stream_matrix(41_000, shape["n_features"], seed=8, missing_rate=0.01)
    s0, v0 = plan.score(X)
    for flags in (0x400, 0x800, 0xC00, 0x4000):  # store_hidden_t on the K = 64 layer / on gemm8 / on both;
        # 0x4000: the K = 64 layer's row segments with ordinary instead of non-temporal stores
        plan.gemm_flags = flags
        try:
            s1, v1 = plan.score(X)
        finally:
            plan.gemm_flags = 0
        assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()]), hex(flags)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,rows,force", [(dict(n_features=32, hidden=(1024, 1024, 512)), 41_000, 0),
                                              (dict(n_features=32, hidden=(1024, 1024, 512)), 300_000, 0),
                                              (dict(n_features=24, hidden=(512, 768, 640), activation="tanh"), 70_000, 0),
                                              (dict(n_features=16, hidden=(512, 512), activation="logistic"), 3_000, 0),
                                              (dict(n_features=300, hidden=(260, 200), activation="tanh"), 50_000, 0x80),
                                              (dict(n_features=16, hidden=(512, 256)), 30_000, 0xC0)],
                         ids=["41k", "300k", "768-odd-tiles", "tiny-grid", "k320-odd-slices", "k64-one-slice"])
def test_persistent_phase_kernel_matches_one_tile_per_workgroup(gpu, shape, rows, force):
    """The persistent tile walk of the phase-interleaved hidden layers (gemm8p_kernel: the slice
    stream continues across tile boundaries, the epilogue runs while the next tile's slices are in
    flight, its stores counted in the next slice's vmcnt) equals gemm8_kernel (flag bit 12, one tile
    per workgroup) bit for bit: more tiles than workgroups (300k rows: 1172 row tiles x 4), a tile
    count that is not a multiple of 8 (the plain round-robin tile list; 768 units = 3 column
    tiles), fewer tiles than CUs (3000 rows), and — the phase kernel forced (bit 7) — an odd slice
    count per tile (300 inputs: K = 320, KT = 5, the buffer parity flips across tile boundaries)
    and one slice per tile (bit 6 + 7 on the K = 64 first layer: KT = 1, every slice is a tile's
    first and last)."""
    c = CompiledPmml.from_string(mlp_pmml(seed=31, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    plan.fuse_head = False
    X = stream_matrix(rows, shape["n_features"], seed=9, missing_rate=0.01)
    plan.gemm_flags = force
    try:
        s0, v0 = plan.score(X)
        for extra in (0x1000,):  # one tile per workgroup
            plan.gemm_flags = force | extra
            s1, v1 = plan.score(X)
            assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()]), hex(extra)
    finally:
        plan.gemm_flags = 0
    n = min(rows, 4000)
    ref, _ = emulate_wide(plan, X[:n])
    got = s0[:n].cpu().numpy().astype(np.float64)
    ok = v0[:n].cpu().numpy().astype(bool)
    np.testing.assert_allclose(got[ok], ref[ok], rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,rows", [(dict(n_features=32, hidden=(1024, 1024)), 300_000),
                                        (dict(n_features=40, hidden=(300, 1024), n_out=3, activation="logistic",
                                              classification=True), 41_000),
                                        (dict(n_features=24, hidden=(512, 768), n_out=4, activation="tanh",
                                              classification=True), 70_000),
                                        (dict(n_features=32, hidden=(512,), n_out=2, classification=True), 50_000)],
                         ids=["reg-300k", "cls3-41k", "cls4-768-odd-tiles", "k64-one-slice"])
def test_persistent_fused_head_matches_one_tile_per_workgroup(gpu, shape, rows):
    """The fused output layer on the persistent tile walk (gemm8p_kernel<true>: head weights and
    biases from LDS, the partial sums in the scratch region, the wave groups re-aligned around the
    exchange barrier) equals gemm8_kernel<true> (flag bit 12) bit for bit — per tile the same
    products in the same order — for n_out 1 to 4 (4: the persistent limit), with a tile count
    that is not a multiple of 8 (768 units = 3 column tiles), and on a K = 64 layer (one slice per
    tile: every slice ends in the head epilogue)."""
    c = CompiledPmml.from_string(mlp_pmml(seed=37, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    assert plan._fused_head()
    X = stream_matrix(rows, shape["n_features"], seed=10, missing_rate=0.01)
    s0, v0 = plan.score(X)
    plan.gemm_flags = 0x1000
    try:
        s1, v1 = plan.score(X)
    finally:
        plan.gemm_flags = 0
    assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()])
    ref, vref = c.score_matrix_oracle(X[:3000])
    v = v0[:3000].cpu().numpy().astype(bool)
    assert (v == vref).all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_persistent_kernels_random_shapes(gpu, seed):
    """Random wide-MLP shapes through the persistent kernels (hidden widths 64-1600, inputs 3-700,
    1-5 outputs, any activation, 1 to 70k rows incl. sub-tile batches), fused head on and off:
    bit-identical to one tile per workgroup (flag bit 12) and within bf16 tolerance of the numpy
    model of the kernels."""
    rng = np.random.default_rng(1000 + seed)
    n_layers = int(rng.integers(1, 4))
    hidden = tuple(int(rng.integers(1, 26)) * 64 for _ in range(n_layers))
    n_out = int(rng.integers(1, 6))
    act = ["rectifier", "tanh", "logistic", "identity"][int(rng.integers(0, 4))]
    n_features = int(rng.integers(3, 700))
    rows = int(rng.choice([1, 255, 257, 3000, 70_000]))
    shape = dict(n_features=n_features, hidden=hidden, n_out=n_out, activation=act,
                 classification=bool(n_out > 1))
    c = CompiledPmml.from_string(mlp_pmml(seed=50 + seed, **shape))
    plan = c.plan(gpu, precision="bf16", mlp_impl="wide")
    X = stream_matrix(rows, n_features, seed=seed, missing_rate=0.2 / n_features)  # ~80 % complete rows
    for fuse in (True, False):
        plan.fuse_head = fuse
        try:
            s0, v0 = plan.score(X)
            plan.gemm_flags = 0x1000
            s1, v1 = plan.score(X)
        finally:
            plan.gemm_flags = 0
            plan.fuse_head = True
        assert torch.equal(v0, v1) and torch.equal(s0[v0.bool()], s1[v1.bool()]), (shape, rows, fuse)
    n = min(rows, 2000)
    ref, ok_ref = emulate_wide(plan, X[:n])
    ok = v0[:n].cpu().numpy().astype(bool)
    assert (ok == ok_ref).all()
    assert ok.any() or n < 10
    got = s0[:n].cpu().numpy().astype(np.float64)
    if not ok.any():
        return
    if shape["classification"]:
        assert (got[ok] == ref[ok]).mean() > 0.97
    else:
        scale = max(1.0, float(np.abs(ref[ok]).max()))
        np.testing.assert_allclose(got[ok], ref[ok], rtol=0, atol=3e-2 * scale)
