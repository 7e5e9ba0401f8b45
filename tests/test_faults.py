"""Fault-injection hooks and the watchdog: fail-load, torn PMML, heartbeat timeout."""

import time

import pytest

from flink_jpmml_amd.api.exceptions import ModelLoadingException
from flink_jpmml_amd.utils.faults import FaultInjector, RankFailure, Watchdog, guarded_collective, set_injector


@pytest.fixture
def faults():
    yield set_injector
    set_injector(None)


def test_parse_env_spec():
    fi = FaultInjector.parse("fail_load=bad.xml; corrupt_pmml=torn ;tear_pmml=gbdt;kill_rank=1@3")
    assert fi.fail_load == ["bad.xml"] and fi.corrupt_pmml == ["torn"] and fi.kill_rank == {1: 3}
    assert fi.tear_pmml == ["gbdt"]
    assert not FaultInjector.parse("").active
    with pytest.raises(ValueError):
        FaultInjector.parse("explode=1")


def test_fail_load_is_fatal_in_static_operator(fixtures_dir, faults):
    from flink_jpmml_amd.api.reader import ModelReader
    from flink_jpmml_amd.stream.operators import EvaluationFunction

    faults(FaultInjector(fail_load=["kmeans"]))
    with pytest.raises(OSError, match="injected"):
        ModelReader(fixtures_dir["kmeans"]).read_bytes()
    fn = EvaluationFunction(ModelReader(fixtures_dir["kmeans"]), lambda e, m: None)
    with pytest.raises(ModelLoadingException):
        fn.open(None)


def test_torn_pmml_never_scores(fixtures_dir, faults):
    from flink_jpmml_amd.api.pmml_model import PmmlModel
    from flink_jpmml_amd.api.reader import ModelReader

    ok = PmmlModel.from_reader(ModelReader(fixtures_dir["kmeans"]))
    assert ok is not None
    faults(FaultInjector(corrupt_pmml=["kmeans"]))
    with pytest.raises(Exception):
        PmmlModel.from_reader(ModelReader(fixtures_dir["kmeans"]))


def test_mid_document_tear_of_large_ensemble_fails_the_job(tmp_path, faults):
    """A torn write inside a 1.3 MB GBDT (the production-size, native-scanner load path): the
    static operator's ``open`` raises ModelLoadingException like the reference's JAXB load
    (`S/api/functions/EvaluationFunction.scala:45-48`), and so does the dynamic operator."""
    from flink_jpmml_amd.api.reader import ModelReader
    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.pmml import flat
    from flink_jpmml_amd.stream.operators import EvaluationFunction

    path = tmp_path / "gbdt_big.pmml"
    path.write_text(synth.gbdt_pmml(n_trees=100, depth=6, n_features=32, seed=3))
    assert path.stat().st_size >= flat.SCAN_MIN_BYTES
    fn = EvaluationFunction(ModelReader(str(path)), lambda e, m: None)
    fn.open(None)  # intact: loads
    faults(FaultInjector(tear_pmml=["gbdt_big"]))
    fn = EvaluationFunction(ModelReader(str(path)), lambda e, m: None)
    with pytest.raises(ModelLoadingException):
        fn.open(None)


def test_watchdog_fires_without_heartbeat():
    fired = []
    with Watchdog(0.2, on_timeout=lambda: fired.append(time.monotonic())) as wd:
        for _ in range(6):  # kicked: no fire
            time.sleep(0.05)
            wd.kick()
        assert not fired
        time.sleep(0.5)
    assert wd.fired and len(fired) == 1


def test_guarded_collective_wraps_peer_errors():
    def boom():
        raise RuntimeError("Connection closed by peer")

    with pytest.raises(RankFailure) as ei:
        guarded_collective(boom, what="all-gather")
    assert isinstance(ei.value.__cause__, RuntimeError)
    assert guarded_collective(lambda x: x + 1, 1) == 2
