"""NeuralNetwork on the MI355X: the persistent panel-ring MFMA kernel (fp32 exact default, bf16
opt-in) on many row tiles per workgroup, and the GEMM path for networks beyond the fused kernel
(1024-unit layers, 10 layers) — all against the float64 oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np(plan, X):
    s, v = plan.score(X)
    return s.cpu().numpy(), v.cpu().numpy()


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-5), ("bf16", 3e-2)])
def test_mlp_64_256_256_1_many_tiles(gpu, precision, tol):
    """The BASELINE config-4 shape over 300K rows (>= 4 row tiles per persistent workgroup, the
    panel ring wraps across tiles), plus rows with a missing input."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.nn_plans import MlpPlan

    c = CompiledPmml.from_string(mlp_pmml(n_features=64, hidden=(256, 256), n_out=1, seed=3))
    plan = c.plan(gpu, precision=precision)
    assert isinstance(plan, MlpPlan) and plan.contiguous == 1 and plan.n_panels == 17
    X = stream_matrix(300_000, 64, seed=11)
    nan_rows = [7, 123_456, 299_999]
    X[nan_rows, [1, 63, 0]] = np.nan
    s, v = _np(plan, X)
    # the per-connection oracle is slow: check every 97th row (all tiles, both lane halves) + the NaN rows
    idx = np.union1d(np.arange(0, len(X), 97), nan_rows)
    s, v = s[idx], v[idx]
    ref, vref = c.score_matrix_oracle(X[idx])
    assert (v == vref).all() and not v[np.searchsorted(idx, nan_rows)].any()
    scale = max(1.0, float(np.max(np.abs(ref[vref]))))
    assert np.max(np.abs(s[v] - ref[v])) < tol * scale


def test_mlp_default_precision_is_fp32(gpu):
    from flink_jpmml_amd.bench.synth import mlp_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(mlp_pmml(n_features=8, hidden=(32,), n_out=1, seed=1))
    assert c.plan(gpu).bf16 == 0 and c.plan(gpu, precision="bf16").bf16 == 1


def test_mlp_gathered_inputs_and_classification(gpu):
    """Gathered inputs (21 inputs do not fill the padded k-steps: per-element index loads) and a softmax
    output layer with 7 classes."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    txt = mlp_pmml(n_features=21, hidden=(50, 33), n_out=7, seed=5, activation="tanh", classification=True)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    assert plan.contiguous == 0  # 21 inputs pad to 22 (fp32) -> gathered loads
    X = stream_matrix(40_000, 21, seed=2)
    s, v = _np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and (s == ref).mean() > 0.9999


@pytest.mark.parametrize("impl", ["auto", "gemm"])
@pytest.mark.parametrize("hidden", [(1024,), (64,) * 9])
def test_mlp_beyond_fused_kernel_runs_on_device(gpu, hidden, impl):
    """A 1024-unit layer and a 10-layer network exceed the fused kernel's registers / LDS: under
    the default fp32 policy they run on the fused GEMM's exact-fp32 MFMA variant (WideMlpPlan);
    ``mlp_impl="gemm"`` forces per-layer library GEMMs. Never on the host."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.nn_plans import GemmMlpPlan, WideMlpPlan

    c = CompiledPmml.from_string(mlp_pmml(n_features=32, hidden=hidden, n_out=1, seed=7))
    plan = c.plan(gpu, mlp_impl=impl)
    assert isinstance(plan, WideMlpPlan if impl == "auto" else GemmMlpPlan) and plan.bf16 == 0
    X = stream_matrix(8192, 32, seed=3)
    X[3, 4] = np.nan
    s, v = _np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all() and not v[3]
    scale = max(1.0, float(np.max(np.abs(ref[vref]))))
    assert np.max(np.abs(s[v] - ref[v])) < 1e-3 * scale


@pytest.mark.parametrize("kernel", ["reg", "panel"])
@pytest.mark.parametrize("shape", [
    dict(n_features=64, hidden=(256, 256), n_out=1, activation="rectifier"),     # BASELINE config 4
    dict(n_features=32, hidden=(100,), n_out=1, activation="logistic"),          # 1 hidden layer, partial tile
    dict(n_features=21, hidden=(50, 33), n_out=7, activation="tanh", classification=True),  # gathered, softmax
    dict(n_features=130, hidden=(256, 64), n_out=1, activation="rectifier"),     # k0 > 64: no prefetch
])
def test_mlp_bf16_kernels_vs_oracle(gpu, kernel, shape):
    """Both bf16 kernels (register-weight and panel-ring) on several shapes over a row count that is
    not a multiple of either kernel's block, with missing inputs, against the float64 oracle."""
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(mlp_pmml(seed=4, **shape))
    plan = c.plan(gpu, precision="bf16")
    plan.set_kernel(kernel)
    assert plan.reg_kernel == (1 if kernel == "reg" else 0)
    n = 70_001
    X = stream_matrix(n, shape["n_features"], seed=9)
    nan_rows = [0, 127, 128, 40_000, n - 1]
    X[nan_rows, 3] = np.nan
    s, v = _np(plan, X)
    idx = np.union1d(np.arange(0, n, 13), nan_rows)
    ref, vref = c.score_matrix_oracle(X[idx])
    s, v = s[idx], v[idx]
    assert (v == vref).all() and not v[np.searchsorted(idx, nan_rows)].any()
    if shape.get("classification"):
        assert (s[v] == ref[v]).mean() > 0.97
    else:
        scale = max(1.0, float(np.max(np.abs(ref[vref]))))
        assert np.max(np.abs(s[v] - ref[v])) < 3e-2 * scale
