"""The native streaming TreeModel reader (load models of the size the reference
advertises, `README.md:239-242`). Every document parsed through the scanner must give the same IR,
the same oracle scores and the same lowered ensemble as the ordinary parser."""

import xml.etree.ElementTree as ET

import numpy as np
import pytest

from flink_jpmml_amd.bench import synth
from flink_jpmml_amd.pmml import flat, parser
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.utils.metrics import METRICS


@pytest.fixture
def scan_everything(monkeypatch):
    monkeypatch.setattr(flat, "SCAN_MIN_BYTES", 0)


def _both(text):
    ref = parser.parse_element(ET.fromstring(text))
    doc = parser.parse_string(text)
    return doc, ref


def _trees(doc):
    return [m for m in parser.iter_models(doc) if hasattr(m, "flat")]


DOCS = {
    "gbdt": lambda: synth.gbdt_pmml(n_trees=40, depth=5, n_features=8, seed=1),
    "gbdt_binary": lambda: synth.gbdt_pmml(n_trees=30, depth=4, n_features=8, seed=2, objective="binary"),
    "rf": lambda: synth.random_forest_pmml(n_trees=25, depth=7, n_features=8, n_classes=3, seed=3),
    "rf_null": lambda: synth.random_forest_pmml(n_trees=10, depth=5, n_features=8, seed=4,
                                                missing_strategy="nullPrediction"),
    "segmented": lambda: synth.segmented_pmml("selectFirst", classification=True, seed=5),
}


@pytest.mark.parametrize("name", sorted(DOCS))
def test_scanned_ir_equals_dom_ir(scan_everything, name):
    text = DOCS[name]()
    doc, ref = _both(text)
    flats = [m for m in _trees(doc) if m.flat is not None]
    assert flats, "the scanner did not run"
    assert doc == ref  # materialised lazily from the arrays: same nodes, predicates, distributions


@pytest.mark.parametrize("name", sorted(DOCS))
def test_scanned_model_scores_and_lowers_like_dom(scan_everything, name):
    from flink_jpmml_amd.runtime.plans import NotLowerable, ensemble_spec

    text = DOCS[name]()
    before = METRICS.counters.get("pmml.flat_materialized_nodes", 0)
    c = CompiledPmml.from_string(text.encode())
    ref = CompiledPmml(parser.parse_element(ET.fromstring(text)))
    try:
        spec = ensemble_spec(c)
    except NotLowerable:
        spec = None
    if name != "segmented":  # plain ensembles lower straight from the arrays
        assert METRICS.counters.get("pmml.flat_materialized_nodes", 0) == before
    X = synth.stream_matrix(3000, len(c.active_fields), seed=9, missing_rate=0.05)
    s1, v1 = c.score_matrix_oracle(X)
    s2, v2 = ref.score_matrix_oracle(X)
    assert (v1 == v2).all()
    np.testing.assert_array_equal(s1[v1], s2[v2])
    if spec is not None:
        spec2 = ensemble_spec(ref)
        assert len(spec.trees) == len(spec2.trees) and spec.weights == spec2.weights
        for a, b in zip(spec.trees, spec2.trees):
            assert a.depth == b.depth and a.null_missing == b.null_missing
            assert sorted(a.leaf_value[a.feature < 0].tolist()) == sorted(b.leaf_value[b.feature < 0].tolist())
            assert sorted(zip(a.feature[a.feature >= 0].tolist(), a.threshold[a.feature >= 0].tolist())) == \
                sorted(zip(b.feature[b.feature >= 0].tolist(), b.threshold[b.feature >= 0].tolist()))


def test_categorical_set_predicates_through_scanner(scan_everything):
    """SimpleSetPredicate bodies travel as raw spans and are parsed on materialisation; the
    membership-column lowering takes the object path and matches the oracle."""
    from test_derive import categorical_tree_doc, cat_inputs

    text = categorical_tree_doc("defaultChild")
    doc, ref = _both(text)
    assert doc.models[0].flat is not None and doc.models[0].flat.raw
    assert doc == ref
    c = CompiledPmml.from_string(text)
    X = cat_inputs()
    s1, v1 = c.score_matrix_oracle(X)
    s2, v2 = CompiledPmml.from_string(text.replace("<PMML ", "<PMML  ")).score_matrix_oracle(X)
    assert (v1 == v2).all() and np.array_equal(s1[v1], s2[v2])


def test_prefixed_namespace_and_entities(scan_everything):
    """``pmml:`` prefixes, comments, entity references and Extension elements inside nodes."""
    text = ('<?xml version="1.0"?><!-- big model -->'
            '<pmml:PMML xmlns:pmml="http://www.dmg.org/PMML-4_4" version="4.4"><pmml:DataDictionary>'
            '<pmml:DataField name="x&amp;y" optype="continuous" dataType="double"/>'
            '<pmml:DataField name="t" optype="continuous" dataType="double"/></pmml:DataDictionary>'
            '<pmml:TreeModel functionName="regression" missingValueStrategy="defaultChild">'
            '<pmml:MiningSchema><pmml:MiningField name="t" usageType="target"/>'
            '<pmml:MiningField name="x&amp;y"/></pmml:MiningSchema>'
            '<pmml:Node id="r" defaultChild="a"><pmml:True/><pmml:Extension name="e"><X/></pmml:Extension>'
            '<pmml:Node id="a" score="1.5"><pmml:SimplePredicate field="x&amp;y" operator="lessThan" value="&#48;.5"/>'
            '</pmml:Node><!-- c --><pmml:Node id="b" score="-2"><pmml:CompoundPredicate booleanOperator="or">'
            '<pmml:SimplePredicate field="x&amp;y" operator="greaterOrEqual" value="0.5"/><pmml:True/>'
            '</pmml:CompoundPredicate></pmml:Node></pmml:Node></pmml:TreeModel></pmml:PMML>')
    doc, ref = _both(text)
    assert doc.models[0].flat is not None
    assert doc == ref
    assert doc.models[0].root.children[0].predicate.value == "0.5"


def test_scanner_declines_embedded_models(scan_everything):
    text = ('<PMML xmlns="http://www.dmg.org/PMML-4_4" version="4.4"><DataDictionary>'
            '<DataField name="x" optype="continuous" dataType="double"/></DataDictionary>'
            '<TreeModel functionName="regression"><MiningSchema><MiningField name="x"/></MiningSchema>'
            '<Node><True/><Regression/></Node></TreeModel></PMML>')
    assert flat.scan_document(text.encode()) is None  # the ordinary parser reports it


def test_large_forest_loads_fast_and_lean(tmp_path):
    """A ~40 MB, 60-tree depth-14 forest (the 214 MB / 300-tree case scaled 1/5) parses through
    the scanner in a fraction of the DOM path's time and lowers without materialising nodes."""
    import time

    from flink_jpmml_amd.runtime.plans import ensemble_spec

    text = synth.random_forest_pmml(n_trees=60, depth=14, n_features=32, n_classes=3, seed=1)
    data = text.encode()
    del text
    before = METRICS.counters.get("pmml.flat_materialized_nodes", 0)
    t0 = time.perf_counter()
    c = CompiledPmml.from_string(data)
    spec = ensemble_spec(c)
    dt = time.perf_counter() - t0
    assert len(spec.trees) == 60 and max(t.depth for t in spec.trees) == 14
    assert METRICS.counters.get("pmml.flat_materialized_nodes", 0) == before
    assert dt < 4.0, dt  # the DOM path needs ~8 s for this document
