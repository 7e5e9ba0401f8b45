"""PMML 4.4 built-in functions in the host expression engine (`pmml/fields.py::eval_expression`):
erf, the standard and general normal CDF / PDF / IDF, hypot, atan2 and the sample stdev, against
scipy / numpy. Missing arguments propagate (stdev: over the present values, ≥ 2 needed). erf, the
standard-normal trio, hypot and atan2 also have derive-kernel opcodes (`tests/test_derive.py`);
the three-argument normal functions and stdev keep derived fields on the host path."""

import math

import numpy as np
import pytest
from scipy import stats
from scipy.special import erf

from flink_jpmml_amd.pmml import ir
from flink_jpmml_amd.pmml.fields import Columns, eval_expression


def _cols(**cols):
    from flink_jpmml_amd.bench.synth import gbdt_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    schema = CompiledPmml.from_string(gbdt_pmml(n_trees=1, depth=1, n_features=1)).schema
    n = len(next(iter(cols.values())))
    return Columns(schema, n, {k: np.asarray(v, dtype=np.float64) for k, v in cols.items()})


def _apply(fn, *names):
    return ir.Apply(fn, [ir.FieldRef(n) for n in names])


X = [-2.5, -0.3, 0.0, 0.7, 1.9, math.nan]
P = [0.01, 0.2, 0.5, 0.8, 0.99, math.nan]


@pytest.mark.parametrize("fn,ref", [
    ("erf", lambda x: erf(x)),
    ("stdNormalCDF", lambda x: stats.norm.cdf(x)),
    ("stdNormalPDF", lambda x: stats.norm.pdf(x)),
])
def test_unary(fn, ref):
    out = eval_expression(_apply(fn, "x"), _cols(x=X))
    np.testing.assert_allclose(out[:-1], ref(np.array(X[:-1])), rtol=1e-12, atol=1e-15)
    assert math.isnan(out[-1])


def test_std_normal_idf():
    out = eval_expression(_apply("stdNormalIDF", "p"), _cols(p=P))
    np.testing.assert_allclose(out[:-1], stats.norm.ppf(P[:-1]), rtol=1e-12)


def test_normal_family():
    c = _cols(x=X, m=[0.5] * 6, s=[2.0] * 6, p=P)
    np.testing.assert_allclose(eval_expression(_apply("normalCDF", "x", "m", "s"), c)[:-1],
                               stats.norm.cdf(X[:-1], 0.5, 2.0), rtol=1e-12)
    np.testing.assert_allclose(eval_expression(_apply("normalPDF", "x", "m", "s"), c)[:-1],
                               stats.norm.pdf(X[:-1], 0.5, 2.0), rtol=1e-12)
    np.testing.assert_allclose(eval_expression(_apply("normalIDF", "p", "m", "s"), c)[:-1],
                               stats.norm.ppf(P[:-1], 0.5, 2.0), rtol=1e-12)


def test_hypot_atan2():
    c = _cols(a=[3.0, -1.0, 0.0], b=[4.0, 1.0, -2.0])
    np.testing.assert_allclose(eval_expression(_apply("hypot", "a", "b"), c), [5.0, math.sqrt(2), 2.0])
    np.testing.assert_allclose(eval_expression(_apply("atan2", "a", "b"), c), np.arctan2([3.0, -1.0, 0.0],
                                                                                         [4.0, 1.0, -2.0]))


def test_stdev_sample():
    c = _cols(a=[1.0, 2.0, math.nan, math.nan], b=[3.0, math.nan, math.nan, 5.0], d=[5.0, 4.0, math.nan, math.nan])
    out = eval_expression(_apply("stdev", "a", "b", "d"), c)
    assert out[0] == pytest.approx(np.std([1, 3, 5], ddof=1))
    assert out[1] == pytest.approx(np.std([2, 4], ddof=1))
    assert math.isnan(out[2]) and math.isnan(out[3])  # none / one present value
