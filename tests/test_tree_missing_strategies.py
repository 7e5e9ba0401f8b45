"""TreeModel ``missingValueStrategy`` = ``weightedConfidence`` / ``aggregateNodes`` (classification):
at the first UNKNOWN child the row is scored down that child and every sibling not FALSE,
recursively; weightedConfidence weights the siblings' confidences by recordCount / parent's,
aggregateNodes sums the reached leaves' record counts. Parity unpinned (no JPMML here): the expected
values are computed by hand from the PMML 4.4 text. Device: the GENERAL tree layout runs the same
mixture (``tree.hip::gen_mixture``; its numpy twin is checked here, the kernel in
``tests/test_mixture_gpu.py``)."""

import math

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _doc(strategy: str, no_true: str = "returnNullPrediction") -> str:
    def leaf(nid, pred, n, yes, no):
        return (f'<Node id="{nid}" score="{"yes" if yes >= no else "no"}" recordCount="{n}">{pred}'
                f'<ScoreDistribution value="yes" recordCount="{yes}"/>'
                f'<ScoreDistribution value="no" recordCount="{no}"/></Node>')

    a1 = leaf("A1", '<SimplePredicate field="y" operator="lessThan" value="0"/>', 30, 25, 5)
    a2 = leaf("A2", '<SimplePredicate field="y" operator="greaterOrEqual" value="0"/>', 30, 15, 15)
    b = leaf("B", '<SimplePredicate field="x" operator="greaterOrEqual" value="0"/>', 40, 10, 30)
    return f"""<?xml version="1.0"?>
<PMML xmlns="http://www.dmg.org/PMML-4_4" version="4.4">
 <Header/>
 <DataDictionary numberOfFields="3">
  <DataField name="x" optype="continuous" dataType="double"/>
  <DataField name="y" optype="continuous" dataType="double"/>
  <DataField name="t" optype="categorical" dataType="string"><Value value="yes"/><Value value="no"/></DataField>
 </DataDictionary>
 <TreeModel functionName="classification" missingValueStrategy="{strategy}" noTrueChildStrategy="{no_true}">
  <MiningSchema><MiningField name="t" usageType="target"/><MiningField name="x"/><MiningField name="y"/></MiningSchema>
  <Node id="root" score="yes" recordCount="100"><True/>
   <ScoreDistribution value="yes" recordCount="50"/><ScoreDistribution value="no" recordCount="50"/>
   <Node id="A" score="yes" recordCount="60"><SimplePredicate field="x" operator="lessThan" value="0"/>
    <ScoreDistribution value="yes" recordCount="40"/><ScoreDistribution value="no" recordCount="20"/>
    {a1}{a2}
   </Node>
   {b}
  </Node>
 </TreeModel>
</PMML>"""


NAN = math.nan
ROWS = np.array([[-1.0, -1.0], [-1.0, 1.0], [1.0, 5.0], [NAN, -1.0], [NAN, 1.0], [-1.0, NAN], [NAN, NAN]])

# P(yes) per row, by hand
WEIGHTED = [25 / 30, 0.5, 0.25,
            0.6 * 25 / 30 + 0.4 * 0.25,          # x missing, y < 0: A (-> A1) weight 60/100, B 40/100
            0.6 * 0.5 + 0.4 * 0.25,              # x missing, y >= 0: A (-> A2), B
            0.5 * 25 / 30 + 0.5 * 0.5,           # y missing under A: A1, A2 each 30/60
            0.6 * (0.5 * 25 / 30 + 0.5 * 0.5) + 0.4 * 0.25]
AGGREGATE = [25 / 30, 0.5, 0.25,
             (25 + 10) / 70, (15 + 10) / 70, (25 + 15) / 60, (25 + 15 + 10) / 100]


@pytest.mark.parametrize("strategy,expected", [("weightedConfidence", WEIGHTED), ("aggregateNodes", AGGREGATE)])
def test_sibling_mixture_by_hand(strategy, expected):
    c = CompiledPmml.from_string(_doc(strategy))
    res = c.result(ROWS)
    assert list(res.categories) == ["yes", "no"]
    assert res.valid.all()
    np.testing.assert_allclose(res.probs[:, 0], expected, rtol=0, atol=1e-12)
    np.testing.assert_allclose(res.probs.sum(axis=1), 1.0, rtol=0, atol=1e-12)
    p = np.asarray(expected)
    sure = np.abs(p - 0.5) > 1e-9
    assert (res.value[sure] == np.where(p[sure] > 0.5, 0, 1)).all()


def test_rows_without_unknowns_keep_their_leaf():
    plain = CompiledPmml.from_string(_doc("none")).result(ROWS[:3])
    mixed = CompiledPmml.from_string(_doc("aggregateNodes")).result(ROWS[:3])
    np.testing.assert_array_equal(plain.probs, mixed.probs)
    np.testing.assert_array_equal(plain.value, mixed.value)


def test_regression_trees_reject_the_strategies():
    from flink_jpmml_amd.api.exceptions import UnsupportedFeatureException

    doc = _doc("weightedConfidence").replace('functionName="classification"', 'functionName="regression"')
    with pytest.raises(UnsupportedFeatureException):
        CompiledPmml.from_string(doc).result(ROWS)


def _emulate(c, X):
    """(labels, probs, valid) of the GENERAL layout's numpy twin (tree.hip gen_walk + gen_mixture)."""
    from flink_jpmml_amd.runtime.general_tree import emulate_general, pack_general
    from flink_jpmml_amd.runtime.plans import TreePlan

    spec = TreePlan._general_spec(c)
    packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
    acc = emulate_general(packed, X, spec.P, len(spec.trees))
    valid = ~np.isnan(acc).any(axis=1)
    a = spec.epi.get("a", 1.0)
    return np.argmax(np.nan_to_num(acc), axis=1), acc * a, valid


@pytest.mark.parametrize("strategy,expected", [("weightedConfidence", WEIGHTED), ("aggregateNodes", AGGREGATE)])
@pytest.mark.parametrize("no_true", ["returnNullPrediction", "returnLastPrediction"])
def test_device_lowering_mixes_siblings(strategy, expected, no_true):
    """Round 6: both strategies lower to the GENERAL layout's sibling mixture
    (tree.hip::gen_mixture); its numpy twin reproduces the hand-computed probabilities."""
    from flink_jpmml_amd.runtime.plans import TreePlan, compile_plan, lowering_dry_run

    c = CompiledPmml.from_string(_doc(strategy, no_true))
    with lowering_dry_run():
        plan = compile_plan(c, "cpu")
    assert isinstance(plan, TreePlan) and plan.layout == "general" and plan.mix_mass is not None
    lab, probs, valid = _emulate(c, ROWS.astype(np.float32).astype(np.float64))
    assert valid.all()
    np.testing.assert_allclose(probs[:, 0], expected, rtol=0, atol=1e-6)
