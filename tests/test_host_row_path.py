"""Host per-record ``predict`` through the 1-row batch oracle (``PmmlModel._predict_one_host``)
must give the per-record pipeline's Prediction (`S/api/PmmlModel.scala:109-119`) on every fixture
and input shape, and must step aside when a subclass replaces a pipeline stage."""

import numpy as np

from flink_jpmml_amd import DenseVector, SparseVector
from flink_jpmml_amd.api.pmml_model import PmmlModel
from flink_jpmml_amd.domain.prediction import Score


class _Pipeline(PmmlModel):
    """A replaced stage (here a pass-through) forces the per-record pipeline."""

    def prepare_input(self, input_map, replace_nan=None):
        return super().prepare_input(input_map, replace_nan)


def test_host_row_path_equals_pipeline_on_every_fixture(fixtures_dir):
    checked = numeric = 0
    for name, path in sorted(fixtures_dir.items()):
        try:
            fast = PmmlModel.from_path(path)
        except Exception:  # noqa: BLE001 - the deliberately malformed fixtures
            continue
        if fast.is_empty or not fast.active_fields:
            continue
        pipe = _Pipeline(fast.evaluator)
        assert fast._host_row_path() == fast._numeric_inputs() and not pipe._host_row_path()
        numeric += fast._numeric_inputs()
        w = len(fast.active_fields)
        rng = np.random.default_rng(2)
        vecs = [DenseVector(rng.uniform(-1.0, 7.0, size=w)) for _ in range(25)]
        vecs += [DenseVector(np.where(rng.random(w) < 0.3, np.nan, rng.uniform(0, 5, size=w))) for _ in range(10)]
        vecs += [DenseVector(np.array([np.nan] * w)), DenseVector(rng.uniform(0.2, 7.0, size=w + 1)),
                 SparseVector(w, [0], [1.5]), SparseVector(w, [], [])]
        for v in vecs:
            for rn in (None, 0.5):
                a, b = pipe.predict(v, rn), fast.predict(v, rn)
                assert isinstance(a.value, Score) == isinstance(b.value, Score), (name, v, rn)
                if isinstance(a.value, Score):
                    assert a.value.value == b.value.value or (np.isnan(a.value.value) and np.isnan(b.value.value)), \
                        (name, v, rn, a.value.value, b.value.value)
        checked += 1
    assert checked >= 5 and numeric >= 3


def test_host_row_path_is_used_for_conforming_vectors(monkeypatch):
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    m = PmmlModel.from_string(gbdt_pmml(n_trees=20, depth=4, n_features=8, seed=1))
    calls = []
    orig = m.prepare_input
    monkeypatch.setattr(m, "prepare_input", lambda *a, **k: calls.append(1) or orig(*a, **k))
    m.predict(DenseVector(np.linspace(-1, 1, 8)))
    assert not calls  # the row path answered
    m.predict(DenseVector(np.linspace(-1, 1, 9)))  # wrong size: the pipeline reports it
    assert m.predict(DenseVector(np.linspace(-1, 1, 9))).value is not None
