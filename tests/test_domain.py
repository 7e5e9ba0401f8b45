"""Ports of the reference's pure unit specs: ModelIdSpec, PredictionSpec, TargetSpec,
MetadataManagerSpec, ModelsManagerSpec, EvaluatorSpec."""

import pickle
import uuid

import pytest

from flink_jpmml_amd.api import (
    EMPTY_EVALUATOR,
    EmptyEvaluatorException,
    EvaluationException,
    Evaluator,
    InputPreparationException,
    InputValidationException,
    JPMMLExtractionException,
    NoSuchElementException,
    WrongModelIdFormat,
    metadata_manager,
    models_manager,
)
from flink_jpmml_amd.domain import (
    AddMessage,
    DelMessage,
    EmptyScore,
    ModelId,
    ModelInfo,
    Prediction,
    Score,
    ServingMessage,
    Target,
    java_string_hash,
)

NAME = "f5c4e8b3-4a1e-4b3c-9b5e-123456789abc"


# --------------------------------------------------------------------- ModelIdSpec (T/models/core/ModelIdSpec.scala:29-53)
def test_model_id_parses_uuid_and_version():
    mid = ModelId.from_identifier(f"{NAME}_1")
    assert mid == ModelId(NAME, 1)
    assert ModelId.fromIdentifier(f"{NAME}_42").version == 42


@pytest.mark.parametrize("bad", ["not-a-uuid_1", f"{NAME}", f"{NAME}_x", f"{NAME}-1", f"{NAME.upper()}_1", "", f"{NAME}_1_2"])
def test_model_id_rejects_bad_format(bad):
    with pytest.raises(WrongModelIdFormat):
        ModelId.from_identifier(bad)


def test_model_id_hash_code_matches_java_string_hash():
    mid = ModelId(NAME, 7)
    assert mid.java_hash_code == java_string_hash(f"{NAME}_7")
    # known Java values
    assert java_string_hash("") == 0
    assert java_string_hash("a") == 97
    assert java_string_hash("hello") == 99162322
    assert java_string_hash("polygenelubricants") == -2147483648


# --------------------------------------------------------------------- TargetSpec / PredictionSpec
def test_target_score_and_empty():
    assert Target.apply(3.0) == Score(3.0)
    assert Score(3.0).get() == 3.0
    assert Score(3.0).get_or_else(-1.0) == 3.0
    assert EmptyScore.get_or_else(-1.0) == -1.0
    assert EmptyScore.getOrElse(2.0) == 2.0
    with pytest.raises(NoSuchElementException):
        EmptyScore.get()
    assert Target.empty() is EmptyScore
    assert pickle.loads(pickle.dumps(EmptyScore)) is EmptyScore


def test_prediction_from_success():
    assert Prediction.extract_prediction(2.5) == Prediction(Score(2.5))
    assert Prediction.extract_prediction(lambda: 4.0) == Prediction(Score(4.0))


@pytest.mark.parametrize("err", [JPMMLExtractionException("x"), InputPreparationException("x"),
                                 InputValidationException("x"), EvaluationException("x"), TypeError("cast"),
                                 ValueError("nfe"), RuntimeError("any"), EmptyEvaluatorException("e")])
def test_prediction_every_failure_is_empty(err):
    assert Prediction.extract_prediction(err) == Prediction(EmptyScore)

    def boom():
        raise err

    assert Prediction.extract_prediction(boom).value is EmptyScore


def test_prediction_empty_is_shared():
    a = Prediction.extract_prediction(RuntimeError())
    b = Prediction.extract_prediction(ValueError())
    assert a is b


# --------------------------------------------------------------------- EvaluatorSpec (T/api/EvaluatorSpec.scala:35-57)
def test_evaluator_adt():
    ev = Evaluator.apply("model")
    assert ev.model == "model"
    assert ev.get_or_else("other") == "model"
    assert Evaluator.empty() is EMPTY_EVALUATOR
    assert EMPTY_EVALUATOR.get_or_else("d") == "d"
    with pytest.raises(EmptyEvaluatorException):
        EMPTY_EVALUATOR.model
    assert isinstance(EmptyEvaluatorException("x"), NoSuchElementException)


# --------------------------------------------------------------------- MetadataManagerSpec (:47-76)
def test_metadata_add_unknown_inserts_and_known_is_unchanged():
    meta = {}
    m1 = metadata_manager(AddMessage(NAME, 1, "/a.xml", 0), meta)
    assert m1 == {ModelId(NAME, 1): ModelInfo("/a.xml")}
    assert meta == {}  # input untouched
    m2 = metadata_manager(AddMessage(NAME, 1, "/b.xml", 1), m1)
    assert m2 == m1  # same id -> ignored (new version needed)
    m3 = metadata_manager(AddMessage(NAME, 2, "/b.xml", 1), m2)
    assert len(m3) == 2


def test_metadata_del_removes():
    meta = {ModelId(NAME, 1): ModelInfo("/a.xml"), ModelId(NAME, 2): ModelInfo("/b.xml")}
    out = metadata_manager(DelMessage(NAME, 1, 0), meta)
    assert out == {ModelId(NAME, 2): ModelInfo("/b.xml")}
    assert metadata_manager(DelMessage(NAME, 9, 0), out) == out


# --------------------------------------------------------------------- ModelsManagerSpec (:50-70)
def test_models_manager_evicts_only_matching():
    keys = {ModelId(NAME, 1), ModelId(NAME, 2), ModelId(NAME, 3).java_hash_code}
    assert models_manager(DelMessage(NAME, 1, 0), keys) == {ModelId(NAME, 1)}
    assert models_manager(DelMessage(NAME, 3, 0), keys) == {ModelId(NAME, 3).java_hash_code}
    assert models_manager(DelMessage(NAME, 5, 0), keys) == set()
    assert models_manager(AddMessage(NAME, 1, "/x", 0), keys) == set()


# --------------------------------------------------------------------- control wire format
def test_control_messages_pack_roundtrip():
    for m in [AddMessage(NAME, 3, "hdfs://nn/models/a.xml", 123), DelMessage(NAME, 3, 456),
              AddMessage("not-a-uuid", 1, "/p", 0), AddMessage(str(uuid.uuid4()), 2**40, "", -1)]:
        back = ServingMessage.unpack(m.pack())
        assert back == m and type(back) is type(m)
    a = AddMessage(NAME, 1, "/p", 0)
    assert a.model_id == ModelId(NAME, 1) and a.modelId == a.model_id and a.model_info == ModelInfo("/p")


def test_metrics_prometheus_exposition():
    import urllib.request

    from flink_jpmml_amd.utils.metrics import Metrics

    m = Metrics()
    m.inc("scoring.rows_device", 4096)
    m.inc("scoring.empty_score.preparation")
    for v in (1.0, 2.0, 3.0):
        m.observe("scoring.batch_latency_ms", v)
    txt = m.prometheus_text(labels={"rank": "0"})
    assert '# TYPE fja_scoring_rows_device counter' in txt
    assert 'fja_scoring_rows_device{rank="0"} 4096' in txt
    assert 'fja_scoring_batch_latency_ms{rank="0",quantile="0.5"} 2' in txt
    assert 'fja_scoring_batch_latency_ms_count{rank="0"} 3' in txt
    srv = m.serve_prometheus(port=0)
    try:
        port = srv.server_address[1]
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        assert "fja_scoring_rows_device 4096" in body
    finally:
        srv.shutdown()
