"""Example jobs run end to end on CPU (reference `E/*.scala`)."""

from flink_jpmml_amd.domain import Target
from flink_jpmml_amd.examples import jobs
from flink_jpmml_amd.examples.sources import ControlSource, IrisSource, ids_and_paths


def test_quick_and_evaluate(fixtures_dir, tmp_path):
    out = jobs.main(["quick", "--model", fixtures_dir["kmeans"], "--output", str(tmp_path / "q.txt"), "--records", "20",
                     "--rate", "0"])
    assert out == 0
    lines = (tmp_path / "q.txt").read_text().splitlines()
    assert len(lines) == 20 and all(line.startswith("(Prediction(Score(") for line in lines)
    jobs.main(["evaluate", "--model", fixtures_dir["kmeans"], "--output", str(tmp_path / "e.txt"), "--records", "10",
               "--batch-size", "4", "--rate", "0"])
    assert len((tmp_path / "e.txt").read_text().splitlines()) == 10


def test_dynamic_finite(fixtures_dir, tmp_path):
    args = jobs.build_parser().parse_args(["dynamic", "--models", f"{fixtures_dir['kmeans']},{fixtures_dir['kmeans41']}",
                                           "--output", str(tmp_path / "d.txt"), "--gen-policy", "finite",
                                           "--records", "30", "--intervalCheckpoint", "20", "--rate", "200",
                                           "--maxIntervalControlStream", "50",
                                           "--checkpoint-dir", str(tmp_path / "ck")])
    out = jobs.dynamic_evaluate_kmeans(args)
    assert len(out) == 30
    assert all(isinstance(t, Target) for _, t in out)
    assert len((tmp_path / "d.txt").read_text().splitlines()) == 30
    assert (tmp_path / "ck").exists() and any((tmp_path / "ck").iterdir())


def test_checkpoint_example_with_control_file(fixtures_dir, tmp_path):
    cf = tmp_path / "paths.txt"
    cf.write_text(fixtures_dir["kmeans"] + "\n")
    jobs.main(["checkpoint", "--control-file", str(cf), "--output", str(tmp_path / "c.txt"), "--records", "12",
               "--rate", "0"])
    assert len((tmp_path / "c.txt").read_text().splitlines()) == 12


def test_reference_defaults():
    """Defaults are the reference's (`E/util/DynamicParams.scala:38-40`, `E/sources/IrisSource.scala:52`)."""
    args = jobs.build_parser().parse_args(["dynamic", "--models", "a.xml", "--output", "-"])
    assert args.maxIntervalControlStream == 5000 and args.intervalCheckpoint == 1000 and args.rate == 1.0
    assert IrisSource(None, rate=1.0).live and ControlSource({}, "finite", max_interval_ms=5000).live
    # unbounded by default: the jobs run until cancelled (`E/sources/IrisSource.scala:52`)
    assert args.records == 0 and jobs._records(args) is None and args.control_messages is None


def test_sources_policies():
    idp = ids_and_paths(["a.xml", "b.xml"])
    assert len(list(ControlSource(idp, "finite").iterate())) == 2
    assert len(list(ControlSource(idp, "loop", n=5).iterate())) == 5
    assert len(list(ControlSource(idp, "random", n=4).iterate())) == 4
    evs = list(IrisSource(list(idp), n=6).iterate())
    assert len(evs) == 6 and all(e.model_id.endswith("_1") for e in evs)
    assert all(0.2 <= v <= 6.0 for e in evs for v in e.to_vector().data)
    assert list(IrisSource(None, n=2).iterate())[0].model_id is None  # no crash without ids (reference bug)


def test_example_config_flags_and_metrics(fixtures_dir, tmp_path):
    """Config flags reach the job (size-or-time flush under a rate-limited source) and the run's
    metrics are written as JSON."""
    import json

    from flink_jpmml_amd.examples.jobs import main, scoring_config, build_parser

    out, met = tmp_path / "q.txt", tmp_path / "m.jsonl"
    rc = main(["quick", "--model", fixtures_dir["kmeans"], "--output", str(out), "--records", "12",
               "--batch-size", "1024", "--max-batch-latency-ms", "5", "--rate", "400", "--fallback", "error",
               "--metrics-out", str(met)])
    assert rc == 0 and len(out.read_text().splitlines()) == 12
    m = json.loads(met.read_text().splitlines()[-1])
    assert m["counters"].get("batcher.latency_flushes", 0) >= 1  # a 1024 batch never fills: time flushes
    args = build_parser().parse_args(["quick", "--model", "x", "--output", "-", "--precision", "bf16",
                                      "--cache-capacity", "3", "--micro-batch", "4096"])
    cfg = scoring_config(args)
    assert cfg.precision == "bf16" and cfg.cache_capacity == 3 and cfg.micro_batch == 4096
