"""Port of `T/api/PmmlModelSpec.scala` (37 cases) + `T/api/converter/VectorConverterSpec.scala` and
the §4.6 goldens, on the float64 host path (no GPU)."""

import glob
import math
import os

import numpy as np
import pytest

from flink_jpmml_amd.api import (
    DenseVector,
    EmptyEvaluatorException,
    InputPreparationException,
    InputValidationException,
    JPMMLExtractionException,
    ModelReader,
    PmmlModel,
    SparseVector,
)
from flink_jpmml_amd.api.converter import vector_conversion
from flink_jpmml_amd.api.exceptions import ModelLoadingException, PmmlParseError
from flink_jpmml_amd.api.pipeline import FieldValue
from flink_jpmml_amd.domain import EmptyScore, Prediction, Score, Target

KEYS = ["sepal_length", "sepal_width", "petal_length", "petal_width"]


@pytest.fixture(scope="module")
def model(fixtures_dir):
    return PmmlModel.from_reader(ModelReader(fixtures_dir["kmeans"]))


@pytest.fixture(scope="module")
def model_strings(fixtures_dir):
    return PmmlModel.from_path(fixtures_dir["kmeans_stringfields"])


@pytest.fixture(scope="module")
def model_no_output(fixtures_dir):
    return PmmlModel.from_path(fixtures_dir["kmeans_nooutput"])


none_model = PmmlModel.empty()


# ------------------------------------------------------------------ goldens (PmmlModelSpec:50-83)
def test_dense_golden(model):
    assert model.predict(DenseVector(1.0, 1.0, 1.0, 1.0), None) == Prediction(Score(3.0))


def test_sparse_golden(model):
    assert model.predict(SparseVector(4, [0, 1, 2, 3], [1.0, 2.0, 3.0, 4.0]), None) == Prediction(Score(4.0))


def test_sparse_with_replace(model):
    assert model.predict(SparseVector(4, [0, 2], [1.0, 2.0]), 0.0) == Prediction(Score(3.0))


def test_sparse_missing_delegated_to_pmml(model):
    assert model.predict(SparseVector(4, [0, 2], [1.0, 2.0]), None) == Prediction(Score(3.0))


def test_all_ones_sparse(model):
    assert model.predict(SparseVector(4, [0, 1, 2, 3], [1.0] * 4)) == Prediction(Score(3.0))


@pytest.mark.parametrize("vec", [DenseVector(1.0, 2.0, 3.0), DenseVector(1.0, 3.0), DenseVector(1, 3, 2, 4, 5),
                                 SparseVector(2, [0], [1.0]), SparseVector(5, [0, 1, 2, 3], [1.0, 2, 3, 4])])
def test_invalid_size_is_empty(model, vec):
    assert model.predict(vec) == Prediction(Target.empty())


def test_golden_distances(model):
    """Per-cluster squared distances for (1,1,1,1): 64.14 / 45.76 / 22.68 / 31.84."""
    ev = model.compiled.evaluator
    d = ev.distances(np.ones((1, 4)))[0]
    assert np.allclose(d, [64.14, 45.76, 22.68, 31.84], atol=0.01)


# ------------------------------------------------------------------ prepareInput (:87-144)
@pytest.mark.parametrize("vec", [DenseVector(1.0, 1.0, 1.0, 1.0), DenseVector(2.0, -1.0, 3.0, 2.0),
                                 SparseVector(4, [0, 1, 2, 3], [1.0, 2.0, 3.0, 4.0]), SparseVector(4, [0, 2], [1.0, 2.0])])
def test_prepare_input(model, vec):
    inp = model.validate_input(vec)
    out = model.prepare_input(inp, None)
    assert list(out) == KEYS
    for k in KEYS:
        if k in inp:
            assert out[k].value == inp[k] and out[k].encoded == inp[k]
        else:
            assert out[k].value is None and math.isnan(out[k].encoded)


def test_prepare_input_with_replace(model):
    inp = model.validate_input(SparseVector(4, [0, 2], [1.0, 2.0]))
    out = model.prepare_input(inp, 0.0)
    assert [out[k].value for k in KEYS] == [1.0, 0.0, 2.0, 0.0]


def test_prepare_input_string_fields_fail(model_strings):
    inp = model_strings.validate_input(DenseVector(1.0, 4.0, -1.0, 3.0))
    with pytest.raises(InputPreparationException):
        model_strings.prepare_input(inp, None)
    assert model_strings.predict(DenseVector(1.0, 4.0, -1.0, 3.0)).value is EmptyScore


def test_empty_model_raises_everywhere():
    with pytest.raises(EmptyEvaluatorException):
        none_model.prepare_input({"a": 1.0}, None)
    with pytest.raises(EmptyEvaluatorException):
        none_model.validate_input(DenseVector(1.0, 3.0))
    with pytest.raises(EmptyEvaluatorException):
        none_model.extract_target({"PCluster": "1"})
    with pytest.raises(EmptyEvaluatorException):
        none_model.extract_output_fields({})
    with pytest.raises(EmptyEvaluatorException):
        none_model.extract_target_fields({})
    assert none_model.predict(DenseVector(1, 1, 1, 1)) == Prediction(EmptyScore)


# ------------------------------------------------------------------ validateInput (:146-192)
@pytest.mark.parametrize("vec", [DenseVector(1.0, 1.0, 1.0, 1.0), DenseVector(2.0, -1.0, 3.0, 2.0)])
def test_validate_dense(model, vec):
    assert model.validate_input(vec) == dict(zip(KEYS, vec.data.tolist()))


def test_validate_sparse(model):
    assert model.validate_input(SparseVector(4, [0, 1, 2, 3], [1.0, 2.0, 3.0, 4.0])) == dict(zip(KEYS, [1.0, 2, 3, 4]))
    assert model.validate_input(SparseVector(4, [0, 2], [1.0, 2.0])) == {"sepal_length": 1.0, "petal_length": 2.0}


@pytest.mark.parametrize("vec", [DenseVector(1.0, 3.0, 2.0, 4.0, 5.0), SparseVector(5, [0, 1, 2, 3], [1.0, 2, 3, 4]),
                                 DenseVector(1.0, 3.0)])
def test_validate_rejects_size(model, vec):
    with pytest.raises(InputValidationException):
        model.validate_input(vec)


# ------------------------------------------------------------------ extractTarget (:194-250)
def test_extract_string_target(model):
    assert model.extract_target({"PCluster": "x", "clazz": "3.0"}) == 3.0


def test_extract_double_target(model):
    assert model.extract_target({"PCluster": "x", "clazz": 3.0}) == 3.0


def test_extract_missing_target(model):
    with pytest.raises(JPMMLExtractionException):
        model.extract_target({"PCluster": "1"})
    with pytest.raises(JPMMLExtractionException):
        model.extract_target({"clazz": None})


def test_extract_non_numeric_string_is_value_error(model):
    with pytest.raises(ValueError):
        model.extract_target({"clazz": "cluster_a"})


# ------------------------------------------------------------------ extract output / target fields (:252-311)
def test_output_and_target_fields(model, model_no_output):
    res = model.evaluate_input(model.prepare_input(model.validate_input(DenseVector(1, 1, 1, 1))))
    assert dict(model.extract_output_fields(res)).keys() == {"PCluster"}
    assert dict(model.extract_target_fields(res)).keys() == {"clazz"}
    assert res == {"clazz": "3", "PCluster": "3"}
    res2 = model_no_output.evaluate_input(model_no_output.prepare_input(model_no_output.validate_input(
        DenseVector(1, 1, 1, 1))))
    assert dict(model_no_output.extract_output_fields(res2)) == {}


def test_predict_with_outputs(model):
    p = model.predict_with_outputs(DenseVector(1, 1, 1, 1))
    assert p == Prediction(Score(3.0)) and p.outputs == {"PCluster": "3"}


# ------------------------------------------------------------------ prepareAndEmit (:313-325)
def test_prepare_and_emit(model):
    fv = FieldValue(1.0, 1.0, "double", "continuous")
    assert model.prepare_and_emit(fv, "field_1") == ("field_1", fv)
    with pytest.raises(InputPreparationException):
        model.prepare_and_emit(Exception(), "field_1")


# ------------------------------------------------------------------ loader (:327-354)
@pytest.mark.parametrize("name", ["kmeans", "kmeans42", "kmeans41", "kmeans40", "kmeans32", "kmeans_nooutput",
                                  "kmeans_nooutput_notarget", "kmeans_stringfields"])
def test_loads(fixtures_dir, name):
    m = PmmlModel.from_reader(ModelReader(fixtures_dir[name]))
    assert m.model_name == "k-means"


def test_v32_actually_loaded_and_scored(fixtures_dir):
    """The reference maps its 3.2 fixture to the 4.1 file (`T/utils/PmmlLoaderKit.scala:33`);
    we really load PMML 3.2 (clusters named "1".."3" -> entity ids are positions)."""
    m = PmmlModel.from_path(fixtures_dir["kmeans32"])
    assert m.compiled.doc.version == "3.2"
    assert m.predict(DenseVector(5.0, 3.4, 1.5, 0.2)) == Prediction(Score(3.0))


def test_wrong_path_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        PmmlModel.from_reader(ModelReader(str(tmp_path / "nope.xml")))


def test_empty_pmml_raises(fixtures_dir):
    with pytest.raises(PmmlParseError):
        PmmlModel.from_path(fixtures_dir["kmeans_empty"])
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    with pytest.raises(ModelLoadingException):
        CompiledPmml.load(fixtures_dir["kmeans_empty"])


def test_no_target_is_empty(fixtures_dir):
    m = PmmlModel.from_path(fixtures_dir["kmeans_nooutput_notarget"])
    assert m.predict(DenseVector(1, 1, 1, 1)) == Prediction(EmptyScore)


REF = "/root/reference/flink-jpmml-assets/src/main/resources"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference fixtures not mounted")
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(REF, "*.xml"))))
def test_reference_fixture_files(path):
    """Parse the reference's own PMML assets (read-only, data files) and check the goldens."""
    name = os.path.basename(path)
    if name == "kmeans_empty.xml":
        with pytest.raises(PmmlParseError):
            PmmlModel.from_path(path)
        return
    m = PmmlModel.from_path(path)
    p = m.predict(DenseVector(1.0, 1.0, 1.0, 1.0))
    if name in ("kmeans_nooutput_notarget.xml", "kmeans_stringfields.xml"):
        assert p == Prediction(EmptyScore)
    else:
        assert p == Prediction(Score(3.0))
    if name == "kmeans.xml":
        assert m.predict(SparseVector(4, [0, 1, 2, 3], [1.0, 2.0, 3.0, 4.0])) == Prediction(Score(4.0))


# ------------------------------------------------------------------ VectorConverterSpec (:40-80)
def test_converter_dense_sparse_and_order(model):
    ev = model.evaluator
    assert list(vector_conversion(DenseVector(1, 2, 3, 4), ev)) == KEYS
    assert vector_conversion(DenseVector(1, 2), ev) == {"sepal_length": 1.0, "sepal_width": 2.0}  # partial map
    assert vector_conversion(SparseVector(4, [1, 3], [5.0, 6.0]), ev) == {"sepal_width": 5.0, "petal_width": 6.0}
    assert vector_conversion(SparseVector(4, [], []), ev) == {}


# ------------------------------------------------------------------ batch API == per-record API
def test_predict_vectors_matches_predict(model):
    vecs = [DenseVector(1, 1, 1, 1), SparseVector(4, [0, 1, 2, 3], [1, 2, 3, 4]), SparseVector(4, [0, 2], [1, 2]),
            DenseVector(1, 2, 3), DenseVector(6.9, 3.1, 5.8, 2.1), SparseVector(4, [], [])]
    batch = model.predict_vectors(vecs)
    assert batch == [model.predict(v) for v in vecs]
    s, v = model.predict_batch(np.array([[1, 1, 1, 1], [1, 2, 3, 4]], float))
    assert s.tolist() == [3.0, 4.0] and v.all()
