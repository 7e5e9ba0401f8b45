"""CSV parsed on the GPU: ``TextBatchSource(parse="device")`` must give
bit-identical fp32 matrices to the host parser (``native/csrc/ingest.cpp``) on the rounding corpus
of ``test_native_ingest.py`` plus messy lines (CRLF, empty lines, quotes, blanks, missing tokens,
ragged rows, junk, inf / nan spellings, unused and reordered columns, a last line without newline),
across many small chunks."""

import numpy as np
import pytest

from flink_jpmml_amd.bench import synth
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.stream.sources import TextBatchSource

pytestmark = pytest.mark.gpu


def _tokens(rng):
    toks = []
    vals = np.concatenate([rng.standard_normal(3000), rng.standard_normal(500) * 1e6, rng.standard_normal(500) * 1e-6,
                           rng.uniform(-1e30, 1e30, 200)])
    for i, v in enumerate(vals):
        fmt = ("{!r}", "{:.7g}", "{:.9g}", "{:.17g}", "{:.6e}", "{:.3E}")[i % 6]
        toks.append(fmt.format(float(np.float32(v)) if i % 2 else float(v)))
    for _ in range(1500):  # random plain decimals, 1-19 digits, exponents
        nd = int(rng.integers(1, 22))
        digits = "".join(str(int(d)) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        t = digits[:dot] + "." + digits[dot:] if dot < nd else digits
        if rng.random() < 0.3:
            t += f"e{int(rng.integers(-45, 40))}"
        toks.append(("-" if rng.random() < 0.5 else "") + t)
    for v in rng.standard_normal(200).astype(np.float32):  # exact fp32 midpoints
        up = np.nextafter(v, np.float32(np.inf))
        toks.append(repr(float((np.float64(v) + np.float64(up)) / 2)))
    toks += ["16777217", "0.1", "-0.0", "+3.5", "1e-40", "3.4028235e38", "3.5e38", "1.1754944e-38", ".5", "5.",
             "-7e+3", "inf", "-Infinity", "nan", "NaN", "NA", "?", "null", "", " 2.5 ", '"3.25"', "\t-1\t", "abc",
             "1.2.3", "1e", "--1", "0x10", "1_0", "12345678901234567890123"]
    return toks


def _write_csv(path, rng, n_lines=6000):
    toks = _tokens(rng)
    cols = ["junk", "f3", "f0", "extra", "f2", "f1"]  # reordered, with unused columns
    lines = [",".join(cols)]
    for i in range(n_lines):
        k = int(rng.integers(0, 9))
        if k == 0:
            lines.append("")  # empty line: no record
            continue
        row = [toks[int(rng.integers(0, len(toks)))] for _ in range(len(cols))]
        if k == 1:
            row = row[: int(rng.integers(1, len(cols)))]  # ragged: missing trailing columns
        elif k == 2:
            row += ["9", "9"]  # extra columns
        line = ",".join(row)
        if k == 3:
            line += "\r"
        lines.append(line)
    path.write_bytes("\n".join(lines).encode())  # no trailing newline
    return path


def _collect(src):
    import torch

    mats = []
    for b in src.iterate():
        X = b.X
        if isinstance(X, torch.Tensor):
            if X.is_cuda:
                torch.cuda.synchronize()
            X = X.cpu().numpy()
        mats.append(np.asarray(X))
    return np.concatenate(mats) if mats else np.zeros((0, 4), np.float32)


@pytest.mark.parametrize("chunk", [1 << 12, 1 << 16, 1 << 26])
def test_device_parse_bit_identical_to_host(gpu, tmp_path, chunk):
    rng = np.random.default_rng(chunk)
    path = _write_csv(tmp_path / "in.csv", rng)
    model = CompiledPmml.from_string(synth.gbdt_pmml(n_trees=4, depth=3, n_features=4, seed=1))
    host = _collect(TextBatchSource(str(path), model, batch_rows=1000, parse="host"))
    dev_src = TextBatchSource(str(path), model, parse="device", device=gpu, device_chunk_bytes=chunk)
    dev = _collect(dev_src)
    assert host.shape == dev.shape and host.shape[0] > 4000
    nan_h, nan_d = np.isnan(host), np.isnan(dev)
    assert (nan_h == nan_d).all(), np.argwhere(nan_h != nan_d)[:5]
    assert np.array_equal(host[~nan_h].view(np.uint32), dev[~nan_d].view(np.uint32))


def test_device_text_scores_like_host_text(gpu, tmp_path):
    """End to end through the DSL: device-parsed batches (device-resident X, ready event) scored
    by quick_evaluate equal the host-parsed ones."""
    from flink_jpmml_amd import ModelReader
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.stream import StreamExecutionEnvironment

    doc = synth.gbdt_pmml(n_trees=50, depth=5, n_features=8, seed=2)
    mpath = tmp_path / "m.pmml"
    mpath.write_text(doc)
    X = synth.stream_matrix(200_000, 8, seed=3, missing_rate=0.02)
    cpath = tmp_path / "x.csv"
    with open(cpath, "w") as fh:
        fh.write(",".join(f"f{j}" for j in range(8)) + "\n")
        np.savetxt(fh, X, fmt="%.7g", delimiter=",")
    model = CompiledPmml.from_string(doc)
    out = {}
    for mode in ("host", "device"):
        env = StreamExecutionEnvironment(config=ScoringConfig(device=gpu, fallback="error"))
        src = TextBatchSource(str(cpath), model, batch_rows=1 << 16, parse=mode, device=gpu,
                              device_chunk_bytes=4 << 20)
        res = env.add_source(src).quick_evaluate(ModelReader(str(mpath))).collect()
        out[mode] = (np.concatenate([p.scores for p, _ in res]), np.concatenate([p.valid for p, _ in res]))
    assert (out["host"][1] == out["device"][1]).all()
    np.testing.assert_array_equal(out["host"][0][out["host"][1]], out["device"][0][out["device"][1]])


@pytest.mark.parametrize("chunk", [1 << 14, 1 << 26])
def test_zero_copy_mapping_equals_staged_reads(gpu, tmp_path, chunk):
    """The registered-mapping path (DMA straight from the page cache) yields the same batches as
    positional reads into the pinned ring, including the last line without a newline."""
    import torch

    from flink_jpmml_amd.stream.device_text import DeviceTextReader, _mapped, release_mapped

    rng = np.random.default_rng(7)
    path = _write_csv(tmp_path / "zc.csv", rng)
    model = CompiledPmml.from_string(synth.gbdt_pmml(n_trees=4, depth=3, n_features=4, seed=1))
    cols = path.read_bytes().split(b"\n", 1)[0].decode().split(",")
    lo = len(path.read_bytes().split(b"\n", 1)[0]) + 1
    size = path.stat().st_size
    got = {}
    for zc in (False, True):
        r = DeviceTextReader(str(path), model, cols, lo, size, gpu, chunk_bytes=chunk, zero_copy=zc)
        mats = [b.X for b in r]
        torch.cuda.synchronize()
        got[zc] = torch.cat(mats).cpu().numpy()
        if zc:
            assert r.zero_copy_active == (_mapped(str(path), r.lib) is not None)
    release_mapped()
    a, b = got[False], got[True]
    assert a.shape == b.shape and a.shape[0] > 4000
    assert np.array_equal(np.isnan(a), np.isnan(b))
    assert np.array_equal(a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
