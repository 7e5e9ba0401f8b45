"""The reference's per-record call pattern on the device.

``evaluate(reader)(f)`` with ``batch_size=None`` calls ``f(event, model)`` per record and ``f``
calls ``model.predict(vector)`` (`S/package.scala:76-82,111-114`, `S/api/PmmlModel.scala:109-119`).
With the default ``device="auto"`` the operator binds the model to the GPU, and ``predict`` scores
the vector as a 1-row batch through the HIP plan — no host float64 walk per record."""

import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_per_record_udf_runs_on_the_device_by_default(gpu, tmp_path):
    from flink_jpmml_amd import DenseVector, ModelReader
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.stream import StreamExecutionEnvironment
    from flink_jpmml_amd.utils.metrics import METRICS

    assert ScoringConfig().device == "auto"
    path = tmp_path / "gbdt.pmml"
    path.write_text(gbdt_pmml(n_trees=1000, depth=6, n_features=32, seed=0))
    n = 20000
    X = stream_matrix(n, 32, seed=5, missing_rate=0.02).astype(np.float64)
    vecs = [DenseVector(r) for r in X]
    env = StreamExecutionEnvironment()  # default config: device="auto" -> this GPU
    before = METRICS.counters.get("scoring.rows_device", 0)
    seen = []
    stamps = []

    def f(v, model):
        seen.append(model.on_device)
        stamps.append(time.perf_counter())
        return model.predict(v).value.get_or_else(float("nan"))

    stream = env.from_collection(vecs).evaluate(ModelReader(str(path)), f)
    out = stream.collect()
    # steady state: the model is read, parsed and lowered before the first call
    rate = (n - 1) / (stamps[-1] - stamps[0])
    assert all(seen) and len(out) == n
    assert METRICS.counters.get("scoring.rows_device", 0) - before >= n  # every record on the GPU
    ref, vref = CompiledPmml.from_string(path.read_text()).score_matrix_oracle(X)
    got = np.array(out)
    assert (np.isfinite(got) == vref).all()
    np.testing.assert_allclose(got[vref], ref[vref], atol=2e-5, rtol=0)
    print(f"per-record device predict, 1000-tree GBDT: {rate:.0f} records/s")
    assert rate >= 5000, rate


def test_per_record_device_predict_matches_host_contract(gpu, fixtures_dir):
    """Device per-record predict equals the host pipeline's Prediction on every fixture model the
    device can lower, including EmptyScore rows (missing values, wrong sizes, sparse vectors)."""
    from flink_jpmml_amd import DenseVector, SparseVector
    from flink_jpmml_amd.api.pmml_model import PmmlModel
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.domain.prediction import Score

    checked = 0
    for name, path in sorted(fixtures_dir.items()):
        try:
            host = PmmlModel.from_path(path)
        except Exception:  # noqa: BLE001 - the deliberately malformed fixtures
            continue
        if host.is_empty or not host.active_fields:
            continue
        dev = PmmlModel.from_path(path).bind(gpu, ScoringConfig(device=gpu, fallback="host"))
        if not dev.on_device:
            continue
        w = len(host.active_fields)
        rng = np.random.default_rng(1)
        vecs = [DenseVector(rng.uniform(0.2, 7.0, size=w)) for _ in range(40)]
        vecs += [DenseVector(np.array([np.nan] * w)), DenseVector(rng.uniform(0.2, 7.0, size=w + 1)),
                 SparseVector(w, [0], [1.5])]
        for v in vecs:
            for rn in (None, 0.5):
                a, b = host.predict(v, rn), dev.predict(v, rn)
                assert isinstance(a.value, Score) == isinstance(b.value, Score), (name, v)
                if isinstance(a.value, Score):
                    assert abs(a.value.value - b.value.value) <= 1e-4 * max(1.0, abs(a.value.value)), (name, v)
        checked += 1
    assert checked >= 3


def test_per_record_device_predict_from_several_threads(gpu, tmp_path):
    """``score_row`` keeps one set of staging buffers per scorer; callers on several threads take
    turns, so every thread gets its own record's score."""
    from concurrent.futures import ThreadPoolExecutor

    from flink_jpmml_amd import DenseVector
    from flink_jpmml_amd.api.pmml_model import PmmlModel
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.config import ScoringConfig

    doc = gbdt_pmml(n_trees=50, depth=5, n_features=16, seed=3)
    m = PmmlModel.from_string(doc).bind(gpu, ScoringConfig(device=gpu, fallback="error"))
    assert m.on_device
    X = stream_matrix(400, 16, seed=8, missing_rate=0.05).astype(np.float64)
    seq = [m.predict(DenseVector(r)).value.get_or_else(float("nan")) for r in X]
    with ThreadPoolExecutor(4) as ex:
        par = list(ex.map(lambda r: m.predict(DenseVector(r)).value.get_or_else(float("nan")), X))
    np.testing.assert_array_equal(np.array(par), np.array(seq))
