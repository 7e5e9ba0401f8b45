"""Literal content of a model fails closed.

The reference parses a predicate's value into the field's data type inside JPMML's evaluation
(`S/api/PmmlModel.scala:159-160`): a threshold that is not a number never scores as one. Here every
value is encoded before the kernels run, so ``pmml/validate.py`` rejects such a document at load
(``PmmlParseError`` → ``ModelLoadingException``), and ``pmml/parser.py`` rejects an ``Array`` whose
``n`` disagrees with its entries.

The structural fuzz (``test_scan_fuzz.py``) mutates markup; this one mutates the *numbers*: a
seeded corpus replaces one predicate value / array entry / array ``n`` at a time with junk
(``abc``, ``1,5``, empty, ``1..2``, ``0x10`` …) or with another number, then loads the document
through both load paths (ElementTree DOM and the native scanner with ``SCAN_MIN_BYTES = 0``):

* junk on a numeric field (and any ``n`` mismatch) must fail the load on BOTH paths;
* anything else must load on both paths and score bit-identically between them (float64 oracle);
* a junk literal on a string field stays a category (a legal document).

The GPU twin (``test_gpu_predicates.py``) scores accepted mutants on the device plans.
"""

from __future__ import annotations

import html
import random
import re

import numpy as np
import pytest

from flink_jpmml_amd.api.exceptions import PmmlParseError
from flink_jpmml_amd.bench import synth
from flink_jpmml_amd.pmml import flat
from flink_jpmml_amd.runtime.compiled import CompiledPmml

JUNK = ["abc", "1,5", "", " ", "1..2", "--1", "0x10", "1e", "1.5.", "+-2", "one", "1 2", "NaN?", "∞"]
NUMBERS = ["0", "-0.0", "1e-3", "2.5", " 0.125 ", "-7", "1E2", "3."]


def documents():
    from test_derive import categorical_tree_doc
    from test_scan_fuzz import HAND, PREFIXED

    return {
        "gbdt": synth.gbdt_pmml(n_trees=3, depth=3, n_features=4, seed=1),
        "rf": synth.random_forest_pmml(n_trees=2, depth=3, n_features=4, n_classes=3, seed=1),
        "categorical": categorical_tree_doc("defaultChild"),
        "hand": HAND,
        "prefixed": PREFIXED,
        "segmented": synth.segmented_pmml("selectFirst", False, n_segments=4, seed=3),
    }


_PRED = re.compile(r'<(?:\w+:)?SimplePredicate field="([^"]*)" operator="(\w+)" value="([^"]*)"')
_ARRAY = re.compile(r'<(?:\w+:)?SimpleSetPredicate field="([^"]*)"[^>]*>\s*<(?:\w+:)?Array ([^>]*)>([^<]*)<')


def sites(text: str):
    """Mutable literal sites: ``(kind, field, start, end)`` spans of the literal text."""
    out = []
    for m in _PRED.finditer(text):
        out.append(("value", html.unescape(m.group(1)), m.start(3), m.end(3)))
    for m in _ARRAY.finditer(text):
        body_start = m.start(3)
        for t in re.finditer(r'"[^"]*"|\S+', m.group(3)):
            out.append(("entry", html.unescape(m.group(1)), body_start + t.start(), body_start + t.end()))
        n = re.search(r'n="(\d+)"', m.group(2))
        if n:
            off = m.start(2) + n.start(1)
            out.append(("n", html.unescape(m.group(1)), off, off + len(n.group(1))))
    return out


def _load(text: str, scan: bool, monkeypatch):
    monkeypatch.setattr(flat, "SCAN_MIN_BYTES", 0 if scan else 1 << 62)
    try:
        return CompiledPmml.from_string(text.encode())
    except PmmlParseError as e:
        return e


def _scores(c: CompiledPmml, seed: int = 0):
    rng = np.random.default_rng(seed)
    X = rng.normal(0, 1, (400, c.n_features))
    if "cat" in c.active_fields:
        X[:, c.active_fields.index("cat")] = rng.integers(0, 6, 400)
    X[rng.random(X.shape) < 0.05] = np.nan
    return c.score_matrix_oracle(X.astype(np.float32).astype(np.float64))


def _numeric(types, fld) -> bool:
    return types.get(fld) in ("integer", "float", "double")


def _is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def check(text: str, kind: str, fld: str, lit: str, types, monkeypatch) -> str:
    dom, scn = _load(text, False, monkeypatch), _load(text, True, monkeypatch)
    must_fail = kind == "n" or (_numeric(types, fld) and not _is_number(lit))
    if kind == "entry" and not lit.strip():
        must_fail = True  # the entry vanished: n no longer matches
    if must_fail:
        assert isinstance(dom, PmmlParseError), (kind, fld, lit)
        assert isinstance(scn, PmmlParseError), (kind, fld, lit)
        return "rejected"
    assert not isinstance(dom, PmmlParseError), (kind, fld, lit, dom)
    assert not isinstance(scn, PmmlParseError), (kind, fld, lit, scn)
    s1, v1 = _scores(dom)
    s2, v2 = _scores(scn)
    assert (v1 == v2).all() and np.array_equal(s1[v1], s2[v2])
    return "accepted"


@pytest.mark.parametrize("name", ["gbdt", "rf", "categorical", "hand", "prefixed", "segmented"])
def test_literal_mutations_fail_closed(monkeypatch, name):
    text = documents()[name]
    types = CompiledPmml.from_string(text).schema.types
    rng = random.Random(f"literal-{name}")
    where = sites(text)
    assert where, name
    seen = {"rejected": 0, "accepted": 0}
    for _ in range(60):
        kind, fld, a, b = rng.choice(where)
        if kind == "n":
            lit = str(int(text[a:b]) + rng.choice([-1, 1, 2]))
        else:
            lit = rng.choice(JUNK if rng.random() < 0.6 else NUMBERS)
            if kind == "entry" and (" " in lit.strip() or lit.startswith('"')):
                lit = "x"
        mutated = text[:a] + lit + text[b:]
        seen[check(mutated, kind, fld, lit, types, monkeypatch)] += 1
    assert seen["rejected"] > 5, seen


def test_verdict_junk_thresholds_are_rejected(tmp_path):
    """value="abc" / "1,5" / "" on a continuous float field loaded and scored every row
    like threshold 0. All three now fail the load (the operators' ModelLoadingException)."""
    from flink_jpmml_amd.api.exceptions import ModelLoadingException

    text = synth.gbdt_pmml(n_trees=2, depth=2, n_features=3, seed=4)
    m = _PRED.search(text)
    for junk in ("abc", "1,5", ""):
        bad = text[:m.start(3)] + junk + text[m.end(3):]
        with pytest.raises(PmmlParseError):
            CompiledPmml.from_string(bad)
        path = tmp_path / "junk.pmml"
        path.write_text(bad)
        with pytest.raises(ModelLoadingException):
            CompiledPmml.load(str(path))


def test_string_field_keeps_arbitrary_literals():
    """On a string field any literal is a category: "1,5" is a (never matching) value, not an error."""
    from test_derive import categorical_tree_doc

    text = categorical_tree_doc().replace('operator="equal" value="a"', 'operator="equal" value="1,5"')
    c = CompiledPmml.from_string(text)
    s, v = _scores(c)
    assert v.any()
    assert c.schema.vocab["cat"]["1,5"] >= 6  # coded past the six declared values


@pytest.mark.parametrize("arr,ok", [('<Array type="real" n="2">0.5 1.5</Array>', True),
                                    ('<Array type="real" n="3">0.5 1.5</Array>', False),
                                    ('<Array type="real" n="1">0.5 1.5</Array>', False),
                                    ('<Array type="real" n="x">0.5 1.5</Array>', False),
                                    ('<Array type="real" n="0"></Array>', True),
                                    ('<Array type="real">0.5 1.5 2.5</Array>', True),
                                    ('<Array type="real" n="2">0.5 abc</Array>', False)])
def test_array_count_and_content(arr, ok):
    from test_scan_fuzz import PREFIXED

    text = re.sub(r"<pmml:Array[^>]*>[^<]*</pmml:Array>", arr.replace("<Array", "<pmml:Array")
                  .replace("</Array>", "</pmml:Array>"), PREFIXED)
    if ok:
        CompiledPmml.from_string(text)
    else:
        with pytest.raises(PmmlParseError):
            CompiledPmml.from_string(text)


@pytest.mark.parametrize("value,ok", [("1", True), ("-1.5", True), ("+.5", True), ("2.", True), ("1e-3", True),
                                      ("6.02E+23", True), ("NaN", True), ("-Infinity", True), (" 7 ", True),
                                      ("inf", False), ("nan", False), ("infinity", False), ("1_000", False),
                                      ("0x1p3", False), ("1.5f", False), ("", False), ("1,5", False)])
def test_literals_follow_java_double_grammar(value, ok):
    """JPMML parses numbers with Double.parseDouble -- Python-only spellings are not
    numbers (Java's type suffixes / hex floats are refused too: no exporter writes them)."""
    from flink_jpmml_amd.pmml.validate import literal_ok

    assert literal_ok("double", value) is ok
