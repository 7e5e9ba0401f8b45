"""Randomized NeuralNetworks on the device (automatic plan choice: fused register / LDS kernel,
wide GEMM kernels or the library GEMM path by shape) vs the float64 oracle: 1-3 hidden layers of
1-300 units, 1-80 inputs, every smooth device activation (identity, logistic, tanh, rectifier,
Gauss, sine, cosine, Elliott, arctan) plus threshold, regression or softmax classification with
2-8 classes, exact fp32 and bf16 precision. Rows: validity equal to the oracle; values within
precision (a small fraction of rows may flip across a threshold / argmax boundary). CPU part: the
lowering decision of every drawn network (no ``NotLowerable``)."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.runtime.compiled import CompiledPmml

ACTS = ["identity", "logistic", "tanh", "rectifier", "Gauss", "sine", "cosine", "Elliott", "arctan", "threshold"]


def _case(seed: int):
    from flink_jpmml_amd.bench.synth import mlp_pmml

    rng = np.random.default_rng(6100 + seed)
    F = int(rng.choice([1, 3, 8, 33, 80]))
    n_hidden = int(rng.integers(1, 4))
    wide = rng.random() < 0.25
    hidden = tuple(int(rng.choice([300, 257, 128]) if wide else rng.integers(1, 48)) for _ in range(n_hidden))
    act = str(rng.choice(ACTS))
    cls = rng.random() < 0.4
    n_out = int(rng.integers(2, 9)) if cls else 1
    prec = "fp32" if seed % 3 else "bf16"
    txt = mlp_pmml(n_features=F, hidden=hidden, n_out=n_out, seed=seed, activation=act, classification=cls)
    return txt, F, cls, prec, act


@pytest.mark.parametrize("seed", range(12))
def test_random_networks_lower(seed):
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    txt, _, _, prec, _ = _case(seed)
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        c.plan("cpu", precision=prec)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(36, 10))
def test_random_networks_on_gpu(gpu, seed):
    from flink_jpmml_amd.bench.synth import stream_matrix

    txt, F, cls, prec, act = _case(seed)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, precision=prec)
    X = stream_matrix(6000, F, seed=seed, missing_rate=0.01)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), (seed, type(plan).__name__)
    if not v.any():
        return
    flip_ok = 0.03 if (act == "threshold" or prec == "bf16") else 0.005
    if cls:
        assert (s[v] == ref[v]).mean() >= 1.0 - flip_ok, (seed, type(plan).__name__, act, prec)
    else:
        tol = 3e-2 if prec == "bf16" else 2e-4
        scale = max(1.0, float(np.abs(ref[v]).max()))
        far = np.abs(s[v] - ref[v]) > tol * scale
        assert far.mean() <= flip_ok, (seed, type(plan).__name__, act, prec, float(far.mean()))
