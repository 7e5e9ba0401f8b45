"""Zero-parse binary record ingest: file (mmap + parallel copy into pinned
buffers, rank-local row ranges) and socket frames, scored through the DSL like any RecordBatch."""

import socket
import threading

import numpy as np

from flink_jpmml_amd import ModelReader
from flink_jpmml_amd.api.pmml_model import PmmlModel
from flink_jpmml_amd.stream import StreamExecutionEnvironment
from flink_jpmml_amd.stream.binary import BinaryBatchSource, read_header, send_binary, write_binary


def test_binary_file_roundtrip_and_scores(fixtures_dir, tmp_path):
    X = np.random.default_rng(1).uniform(0.2, 7.0, size=(10_007, 4)).astype(np.float32)
    path = write_binary(str(tmp_path / "x.fjab"), X)
    assert read_header(path)[:2] == (4, 10_007)
    env = StreamExecutionEnvironment()
    out = env.read_binary_batches(path, batch_rows=1000, threads=3).quick_evaluate(
        ModelReader(fixtures_dir["kmeans"])).collect()
    got = np.concatenate([b.numpy() for _, b in out])
    np.testing.assert_array_equal(got, X)
    assert [b.offset for _, b in out] == list(range(0, 10_007, 1000))
    scores = np.concatenate([p.values(-1) for p, _ in out])
    ref = PmmlModel.from_path(fixtures_dir["kmeans"]).predict(X.astype(np.float64)).values(-1)
    np.testing.assert_array_equal(scores, ref)


def test_binary_file_rank_ranges_cover_every_row_once(tmp_path):
    X = np.arange(4 * 1001, dtype=np.float32).reshape(1001, 4)
    path = write_binary(str(tmp_path / "x.fjab"), X)
    parts = []
    for r in range(4):
        src = BinaryBatchSource(path, batch_rows=128)
        src.open_subtask(r, 4)
        parts.append(np.concatenate([b.numpy() for b in src.iterate()]))
    np.testing.assert_array_equal(np.concatenate(parts), X)
    assert all(abs(len(p) - 250) <= 1 for p in parts)


def test_socket_binary_frames(fixtures_dir):
    X = np.random.default_rng(2).uniform(0.2, 7.0, size=(3000, 4)).astype(np.float32)
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def serve():
        c, _ = srv.accept()
        for i in range(0, 3000, 700):
            send_binary(c, X[i:i + 700])
        send_binary(c, np.zeros((0, 4), np.float32), end=True)
        c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    env = StreamExecutionEnvironment()
    out = env.socket_binary_stream("127.0.0.1", port).quick_evaluate(ModelReader(fixtures_dir["kmeans"])).collect()
    t.join(5)
    srv.close()
    np.testing.assert_array_equal(np.concatenate([b.numpy() for _, b in out]), X)
    assert len(out) == 5


def test_binary_file_parallel_reads_exact_and_truncation_detected(tmp_path):
    """Positional reads by several threads land every row in place (odd row counts, batches that
    do not divide the file, more threads than rows in a batch); a file cut short raises instead
    of yielding a batch with unread rows."""
    import pytest

    X = np.random.default_rng(3).standard_normal((1003, 7)).astype(np.float32)
    path = write_binary(str(tmp_path / "x.fjab"), X)
    for threads, rows in ((1, 1003), (4, 100), (16, 5)):
        src = BinaryBatchSource(path, batch_rows=rows, threads=threads, repeat=2)
        got = np.concatenate([b.X.numpy() for b in src.iterate()])
        np.testing.assert_array_equal(got, np.concatenate([X, X]))
    with open(path, "r+b") as fh:
        fh.truncate(64 + 500 * 7 * 4 + 3)
    with pytest.raises(EOFError):
        list(BinaryBatchSource(path, batch_rows=256, threads=4).iterate())
