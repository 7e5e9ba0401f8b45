"""Native C++ record ingest (``flink_jpmml_amd/native``): delimited text -> the engine's fp32
matrix, checked against numpy / Python parsing and the float64 oracle."""

import numpy as np
import pytest

from flink_jpmml_amd.native import RecordParser, parse_records
from flink_jpmml_amd.runtime.compiled import CompiledPmml


@pytest.fixture(scope="module")
def kmeans(fixtures_dir):
    return CompiledPmml.load(fixtures_dir["kmeans"])


def test_numeric_csv_matches_numpy(kmeans):
    rng = np.random.default_rng(0)
    X = rng.normal(0, 3, (5000, 4)).astype(np.float32)
    text = "\n".join(",".join(repr(float(v)) for v in row) for row in X).encode() + b"\n"
    m = parse_records(kmeans, text, kmeans.active_fields)
    assert m.shape == X.shape and m.dtype == np.float32
    np.testing.assert_array_equal(m, X)


def test_missing_tokens_reordered_and_skipped_columns(kmeans):
    cols = ["id"] + list(reversed(kmeans.active_fields)) + ["extra"]
    text = b"7,4.0,3,,1e0,zz\n8, NA ,?,2.5,-1.25,q\r\n9,1,1,1,1,\n"
    m = parse_records(kmeans, text, cols)
    # active order is the reverse of the file order
    assert m.shape == (3, 4)
    np.testing.assert_array_equal(m[0], [1.0, np.nan, 3.0, 4.0])
    np.testing.assert_array_equal(m[1], [-1.25, 2.5, np.nan, np.nan])
    s, v = kmeans.score_matrix_oracle(m)
    assert v[2] and s[2] == 3.0  # the reference golden (1,1,1,1) -> cluster 3


def test_categorical_codes_and_unknown_tokens():
    from test_derive import categorical_tree_doc

    c = CompiledPmml.from_string(categorical_tree_doc())
    text = b"x,cat\n0.5,a\n-1,f\n2,zz\n,c\n"
    p = RecordParser(c, ["x", "cat"])
    m, used = p.parse(text.split(b"\n", 1)[1])
    vocab = c.schema.values["cat"]
    assert m[0, 1] == vocab.index("a") and m[1, 1] == vocab.index("f")
    assert m[2, 1] == -1.0  # unknown category -> invalid code
    assert np.isnan(m[3, 0]) and m[3, 1] == vocab.index("c")
    s, v = c.score_matrix_oracle(m)
    assert v.tolist()[:3] == [True, True, False]  # "zz" is not a valid value -> returnInvalid


def test_threads_and_partial_lines(kmeans):
    rng = np.random.default_rng(1)
    X = rng.normal(0, 1, (200_000, 4)).astype(np.float32)
    text = "\n".join(",".join(f"{v:.6g}" for v in row) for row in X).encode() + b"\n"
    p1 = RecordParser(kmeans, kmeans.active_fields, threads=1)
    p8 = RecordParser(kmeans, kmeans.active_fields, threads=8)
    a, used_a = p1.parse(text)
    b, used_b = p8.parse(text)
    assert used_a == used_b == len(text) and np.array_equal(a, b)
    np.testing.assert_allclose(a, X, rtol=1e-5)
    # a trailing partial line is left for the next chunk
    cut = len(text) - 7
    m, used = p8.parse(text[:cut])
    assert len(m) == len(X) - 1 and text[used - 1:used] == b"\n"
    # max_rows caps the batch and reports the bytes it covered
    m, used = p8.parse(text, max_rows=1000)
    assert len(m) == 1000 and text[:used].count(b"\n") == 1000


def test_parse_file_chunks(tmp_path, kmeans):
    rng = np.random.default_rng(2)
    X = rng.normal(0, 1, (30_000, 4)).astype(np.float32)
    path = tmp_path / "rec.csv"
    with open(path, "w") as fh:
        fh.write(",".join(kmeans.active_fields) + "\n")
        for row in X:
            fh.write(",".join(repr(float(v)) for v in row) + "\n")
    p = RecordParser(kmeans, kmeans.active_fields)
    got = np.concatenate(list(p.parse_file(str(path), chunk_bytes=50_000)))
    np.testing.assert_array_equal(got, X)


@pytest.mark.parametrize("sanitizer", ["address,undefined", "thread"])
def test_ingest_under_host_sanitizers(tmp_path, sanitizer):
    """the C++ host ingest built with ASan+UBSan / TSan and driven by a standalone
    edge-case harness (exact-size buffers, CRLF, ragged rows, caps inside another thread's range)."""
    import os
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("no g++")
    src = os.path.join(os.path.dirname(__file__), "..", "flink_jpmml_amd", "native", "csrc", "ingest_selftest.cpp")
    exe = str(tmp_path / "selftest")
    subprocess.run(["g++", "-std=c++17", "-g", "-O1", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer",
                    "-pthread", src, "-o", exe], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ingest selftest: ok" in r.stdout


def _f32_correctly_rounded(tok: str) -> np.float32:
    """Exact reference: the fp32 nearest to the decimal token (ties to even), via rationals."""
    from fractions import Fraction

    x = Fraction(tok)
    if x == 0:
        return np.float32(-0.0 if tok.lstrip().startswith("-") else 0.0)
    c = np.float32(float(x))  # within one ulp (the double step can round twice)
    with np.errstate(over="ignore"):
        cands = [np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))]
    cands = [f for f in cands if np.isfinite(f)]
    best = min(cands, key=lambda f: (abs(Fraction(float(f)) - x), int(np.array(f).view(np.uint32)) & 1))
    return np.float32(best)


def test_numeric_tokens_are_correctly_rounded(kmeans):
    """Numeric tokens parse to the correctly rounded fp32 (std::from_chars, no double rounding) for
    shortest reprs, %.7g / %.9g / %.17g, scientific notation, integers and float midpoints —
    checked bit-exactly against an exact rational reference. (A Clinger fast path measured no
    faster than libstdc++'s from_chars on these ~10-character tokens and was dropped.)"""
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.standard_normal(3000), rng.standard_normal(1000) * 1e6,
                           rng.standard_normal(1000) * 1e-6, rng.uniform(-1e30, 1e30, 300)])
    toks = []
    for i, v in enumerate(vals):
        fmt = ("{!r}", "{:.7g}", "{:.9g}", "{:.17g}", "{:.6e}", "{:.3E}")[i % 6]
        toks.append(fmt.format(float(np.float32(v)) if i % 2 else float(v)))
    toks += ["16777217", "16777219", "0.1", "-0.0", "+3.5", "1e22", "1e-22", "123456789012345678",
             "3.4028235e38", "1.1754944e-38", "33554433.0", "0.000001", ".5", "5.", "-7e+3"]
    F = len(kmeans.active_fields)
    toks = toks[: len(toks) // F * F]
    text = "\n".join(",".join(toks[r * F:(r + 1) * F]) for r in range(len(toks) // F)).encode() + b"\n"
    m = parse_records(kmeans, text, kmeans.active_fields).reshape(-1)
    ref = np.array([_f32_correctly_rounded(t) for t in toks], np.float32)
    assert np.array_equal(m.view(np.uint32), ref.view(np.uint32))


def _round_to_f32(s: str) -> np.float32:
    """Correctly rounded decimal -> fp32 (exact rational arithmetic, ties to even)."""
    from fractions import Fraction

    x = Fraction(s)
    if x == 0:
        return np.float32(-0.0) if s.startswith("-") else np.float32(0.0)
    f = np.float32(float(x))  # within one ulp (double rounding)
    best, best_err = None, None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        if not np.isfinite(c):
            continue
        err = abs(Fraction(float(c)) - x)
        if best is None or err < best_err or (err == best_err and int(c.view(np.uint32)) % 2 == 0):
            best, best_err = c, err
    return best


def test_fast_decimal_path_is_correctly_rounded(kmeans):
    """The Clinger fast path of the native parser (plain decimals, <= 19 digits, |exp| <= 22) and
    its from_chars fallback round every token exactly like a correctly rounded decimal->fp32
    conversion — including decimals whose double image sits on an fp32 midpoint."""
    rng = np.random.default_rng(123)
    toks = []
    for _ in range(4000):
        nd = int(rng.integers(1, 20))
        digits = "".join(str(int(d)) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        t = digits[:dot] + "." + digits[dot:] if dot < nd else digits
        if rng.random() < 0.3:
            t += f"e{int(rng.integers(-25, 16))}"
        if rng.random() < 0.5:
            t = "-" + t
        toks.append(t.lstrip(".") if t.startswith(".") and rng.random() < 0.5 else t)
    # exact fp32 midpoints written out (their double images are midpoints too)
    for v in rng.standard_normal(300).astype(np.float32):
        up = np.nextafter(v, np.float32(np.inf))
        mid = (np.float64(v) + np.float64(up)) / 2
        toks.append(repr(float(mid)))
    toks += ["0", "-0.0", "1e-40", "3.4028235e38", "123456789012345678", "0.1", "7.0000005"]
    width = len(kmeans.active_fields)
    lines = [",".join([t] + ["0"] * (width - 1)) for t in toks]
    X = parse_records(kmeans, ("\n".join(lines) + "\n").encode(), kmeans.active_fields)
    got = X[:, 0]
    want = np.array([_round_to_f32(t) for t in toks], dtype=np.float32)
    bad = [(t, g, w) for t, g, w in zip(toks, got, want) if g.view(np.uint32) != w.view(np.uint32)]
    assert not bad, bad[:10]


def test_swar_digit_runs_and_buffer_edges(kmeans):
    """Single-pass numeric fields with SWAR digit runs: integer / fraction runs of 1-20 digits
    (8- and 16-digit run boundaries, > 19 digits through the scalar path), leading zeros, signs,
    exponents, CRLF, a numeric missing token, and fields in the last bytes of the buffer."""
    toks = []
    for n in list(range(1, 21)):
        digits = "".join(str((i * 7 + 3) % 10) for i in range(n))
        toks += [digits, "-" + digits, "0." + digits, digits[: max(1, n // 2)] + "." + digits[n // 2:],
                 "+" + digits + "e-3", "00000" + digits[:6]]
    toks += ["0", "-0", "0.0", "1e22", "1e-22", "123456789012345678", "9007199254740993", "3.4028235e38"]
    rows = [toks[i: i + 4] for i in range(0, len(toks) - 3, 4)]
    text = "\n".join(",".join(r) for r in rows).encode()
    for tail in (b"\n", b"\r\n"):
        m = parse_records(kmeans, text + tail, kmeans.active_fields)
        want = np.array([[np.float32(float(t)) for t in r] for r in rows], dtype=np.float32)
        np.testing.assert_array_equal(m, want)
    # short final line: the SWAR loads must stay inside the buffer (scalar path near the end)
    m = parse_records(kmeans, b"1,2,3,4\n5,6,7,8", kmeans.active_fields)
    np.testing.assert_array_equal(m, [[1, 2, 3, 4], [5, 6, 7, 8]])
    # a numeric missing token keeps its meaning (the single-pass path is off then)
    p = RecordParser(kmeans, kmeans.active_fields, missing=("-999",))
    m, _ = p.parse(b"-999,1.5,-999.5,2\n")
    np.testing.assert_array_equal(m, [[np.nan, 1.5, -999.5, 2.0]])


@pytest.mark.parametrize("use_mmap", [True, False])
@pytest.mark.parametrize("trailing_newline", [True, False])
@pytest.mark.parametrize("chunk,batch_rows", [(64, 7), (1000, 1000), (1 << 20, 100000)])
def test_text_source_window_fills_batches(tmp_path, trailing_newline, chunk, batch_rows, use_mmap):
    """TextBatchSource's reusable read window: lines longer than the window grow it, partial lines
    carry over, batches are filled to ``batch_rows`` across chunks, rank splits cover every row."""
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.stream.sources import TextBatchSource

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=2, depth=2, n_features=4))
    X = stream_matrix(3000, 4, seed=1, missing_rate=0.05)
    path = tmp_path / "x.csv"
    body = "\n".join(",".join("" if np.isnan(v) else f"{v:.9g}" for v in r) for r in X)
    path.write_text("f0,f1,f2,f3\n" + body + ("\n" if trailing_newline else ""))
    for world in (1, 3):
        got = []
        for r in range(world):
            src = TextBatchSource(str(path), c, batch_rows=batch_rows, chunk_bytes=chunk, use_mmap=use_mmap)
            src.open_subtask(r, world)
            bs = list(src.iterate())
            assert all(len(b) == batch_rows for b in bs[:-1])
            got += [b.X.numpy() for b in bs]
        M = np.concatenate(got)
        assert M.shape == X.shape
        np.testing.assert_array_equal(np.isnan(M), np.isnan(X))
        np.testing.assert_allclose(np.nan_to_num(M), np.nan_to_num(X), rtol=1e-7)
