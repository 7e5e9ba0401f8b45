"""Restoring a time-based checkpoint at a different world size (`stream/runtime.py`).

A time-triggered manifest stores one processed cut per rank (`ranks`), because ranks stop at
different offsets. Restoring it at another world size must neither lose nor duplicate records:
shard-mode sources resume at the smallest cut and skip every global offset ``g`` that its old
owner (``g % old_world``) had already processed; replicated sources replay from the smallest cut
(idempotent control messages); rank-local ``parallel`` and ``either`` splits refuse.
"""

from types import SimpleNamespace

import pytest

from flink_jpmml_amd.stream.sources import CollectionSource, SourceReader

N = 40
CUTS = [20, 9]  # old world 2: rank 0 processed evens < 20, rank 1 processed odds < 9


def _unprocessed():
    return [g for g in range(N) if g >= CUTS[g % 2]]


class _NoShard:
    """A pull source without ``iterate_shard`` (read in full, filtered per rank)."""

    def __init__(self, items):
        self.items = items

    def iterate(self):
        return iter(self.items)

    def seek(self, off):
        return iter(self.items[off:])


@pytest.mark.parametrize("new_world", [1, 2, 3, 4])
@pytest.mark.parametrize("strided", [True, False])
def test_shard_restore_at_new_world_size_is_exact(new_world, strided):
    items = list(range(N))
    got = []
    for r in range(new_world):
        src = CollectionSource(items) if strided else _NoShard(items)
        node = SimpleNamespace(source=src, dist_mode="shard")
        rd = SourceReader(node, r, new_world, None, min(CUTS), owner_cuts=CUTS)
        assert rd.chunks(8) is None  # the chunked fast path does not know the cuts
        got.extend(g for g, _ in rd)
    assert sorted(got) == _unprocessed()  # nothing lost
    assert len(got) == len(set(got))  # nothing twice


def test_runtime_rescaled_restore_from_time_manifest(tmp_path, fixtures_dir):
    """End to end: a world-2 time manifest restored by a world-1 job scores exactly the records
    the two old ranks had not processed."""
    from flink_jpmml_amd.stream import FileSink, StreamExecutionEnvironment
    from flink_jpmml_amd.stream.state import CheckpointStorage

    store = CheckpointStorage(str(tmp_path / "ck"))
    manifest = store.write(3, {"trigger": "time", "operators": {},
                               "sources": {"events": {"offset": CUTS[0], "ranks": CUTS}}})
    env = StreamExecutionEnvironment()
    env.from_collection(list(range(N)), uid="events").map(lambda x: [x]).add_sink(FileSink(str(tmp_path / "out")))
    env.execute("rescaled", restore=manifest)
    got = sorted(r[0] for r in FileSink.read(str(tmp_path / "out")))
    assert got == _unprocessed()


def test_either_split_refuses_rescale(tmp_path):
    from flink_jpmml_amd.stream import FileSink, StreamExecutionEnvironment
    from flink_jpmml_amd.stream.state import CheckpointStorage

    store = CheckpointStorage(str(tmp_path / "ck"))
    manifest = store.write(1, {"trigger": "time", "operators": {},
                               "sources": {"events": {"offset": 4, "ranks": [4, 5]}}})
    env = StreamExecutionEnvironment()
    s = env.from_collection(list(range(10)), uid="events")
    s.node.dist_mode = "either"
    s.map(lambda x: [x]).add_sink(FileSink(str(tmp_path / "out")))
    with pytest.raises(RuntimeError, match="world size 2"):
        env.execute("either", restore=manifest)


def test_checkpoint_inside_skip_window_keeps_owner_cuts(tmp_path):
    """restore a world-2 manifest at world 1, take a checkpoint while the reader is still
    inside the old owners' skip window (offset 12 < max cut 20), fail, restore from THAT checkpoint:
    the old cuts must travel in the manifest (``skip_layers``) so elements 12..19 the old rank 0 had
    processed are not scored a second time."""
    from flink_jpmml_amd.stream import FileSink, StreamExecutionEnvironment
    from flink_jpmml_amd.stream.state import CheckpointStorage

    store = CheckpointStorage(str(tmp_path / "ck0"))
    first = store.write(3, {"trigger": "time", "operators": {},
                            "sources": {"events": {"offset": CUTS[0], "ranks": CUTS}}})

    def job(restore, fail_after=None):
        env = StreamExecutionEnvironment()
        env.enable_checkpointing(every_n_records=12, directory=str(tmp_path / "ck"))
        if fail_after is not None:
            env.inject_failure(fail_after)
        env.from_collection(list(range(N)), uid="events").map(lambda x: [x]) \
            .add_sink(FileSink(str(tmp_path / "out")))
        return env.execute("rescaled-twice", restore=restore)

    with pytest.raises(Exception):
        job(first, fail_after=5)
    ck = CheckpointStorage(str(tmp_path / "ck"))
    doc = CheckpointStorage.read(ck.latest())
    assert doc["sources"]["events"]["offset"] == 12
    assert doc["sources"]["events"]["skip_layers"] == [CUTS]
    job(ck.latest())
    got = [r[0] for r in FileSink.read(str(tmp_path / "out"))]
    assert sorted(got) == _unprocessed() and len(got) == len(set(got))
    # past the window the layers are dropped from later manifests
    last = CheckpointStorage.read(CheckpointStorage(str(tmp_path / "ck")).latest())
    assert "skip_layers" not in last["sources"]["events"]


def test_skip_layers_compose():
    """Two rescales: world 2 cuts [20, 9], then world 3 cuts [24, 13, 30] recorded while the first
    window was open. A world-2 restore skips what either layer marks processed."""
    items = list(range(N))
    layers = [CUTS, [24, 13, 30]]
    got = []
    for r in range(2):
        node = SimpleNamespace(source=CollectionSource(items), dist_mode="shard")
        got.extend(g for g, _ in SourceReader(node, r, 2, None, 13, owner_cuts=layers))
    want = [g for g in range(13, N) if not any(g < lay[g % len(lay)] for lay in layers)]
    assert sorted(got) == want and len(got) == len(set(got))
