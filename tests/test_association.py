"""AssociationModel: loads (the reference's JPMML evaluates it), ``predict`` is ``EmptyScore`` (no
target field, `S/api/PmmlModel.scala:167-174`), the rules come out of ``ruleValue`` outputs."""

import math

import numpy as np
import pytest

from flink_jpmml_amd import DenseVector, PmmlModel
from flink_jpmml_amd.domain.prediction import EmptyScore

DOC = """<?xml version="1.0"?>
<PMML version="4.3" xmlns="http://www.dmg.org/PMML-4_3">
 <Header/>
 <DataDictionary numberOfFields="3">
  <DataField name="a" optype="categorical" dataType="integer"><Value value="1"/><Value value="2"/><Value value="3"/><Value value="4"/></DataField>
  <DataField name="b" optype="categorical" dataType="integer"><Value value="1"/><Value value="2"/><Value value="3"/><Value value="4"/></DataField>
  <DataField name="c" optype="categorical" dataType="integer"><Value value="1"/><Value value="2"/><Value value="3"/><Value value="4"/></DataField>
 </DataDictionary>
 <AssociationModel functionName="associationRules" numberOfTransactions="4" minimumSupport="0.5"
   minimumConfidence="0.3" numberOfItems="4" numberOfItemsets="5" numberOfRules="4">
  <MiningSchema><MiningField name="a"/><MiningField name="b"/><MiningField name="c"/></MiningSchema>
  <Output>
   <OutputField name="rec1" feature="ruleValue" ruleFeature="consequent" algorithm="recommendation" rank="1"/>
   <OutputField name="rec2" feature="ruleValue" ruleFeature="consequent" algorithm="recommendation" rank="2"/>
   <OutputField name="excl" feature="ruleValue" ruleFeature="consequent"/>
   <OutputField name="assoc" feature="ruleValue" ruleFeature="rule" algorithm="ruleAssociation"/>
   <OutputField name="conf" feature="ruleValue" ruleFeature="confidence" algorithm="recommendation" dataType="double"/>
   <OutputField name="by_lift" feature="ruleValue" ruleFeature="ruleId" algorithm="recommendation" rankBasis="lift"/>
   <OutputField name="low_support" feature="ruleValue" ruleFeature="support" algorithm="recommendation" rankBasis="support" rankOrder="ascending" dataType="double"/>
   <OutputField name="rid" feature="entityId" algorithm="recommendation"/>
  </Output>
  <Item id="1" value="1"/><Item id="2" value="2"/><Item id="3" value="3"/><Item id="4" value="4"/>
  <Itemset id="1" numberOfItems="1"><ItemRef itemRef="1"/></Itemset>
  <Itemset id="2" numberOfItems="1"><ItemRef itemRef="2"/></Itemset>
  <Itemset id="3" numberOfItems="1"><ItemRef itemRef="3"/></Itemset>
  <Itemset id="4" numberOfItems="2"><ItemRef itemRef="1"/><ItemRef itemRef="3"/></Itemset>
  <Itemset id="5" numberOfItems="1"><ItemRef itemRef="4"/></Itemset>
  <AssociationRule id="r1" support="1.0" confidence="1.0" lift="1.0" antecedent="1" consequent="2"/>
  <AssociationRule id="r2" support="0.5" confidence="0.75" lift="1.5" antecedent="1" consequent="3"/>
  <AssociationRule id="r3" support="0.5" confidence="0.9" lift="1.2" antecedent="4" consequent="5"/>
  <AssociationRule id="r4" support="0.75" confidence="0.6" lift="0.8" antecedent="3" consequent="1"/>
 </AssociationModel>
</PMML>"""


@pytest.fixture(scope="module")
def model():
    return PmmlModel.from_string(DOC)


def test_loads_and_scores_empty_like_the_reference(model):
    assert model.predict(DenseVector(1.0, 3.0, 4.0)).value is EmptyScore
    pb = model.predict(np.array([[1.0, 2.0, 3.0], [4.0, 4.0, 4.0]]))
    assert not pb.valid.any()


def test_rule_outputs(model):
    out = model.predict_with_outputs(DenseVector(1.0, 3.0, float("nan"))).outputs  # basket {1, 3}
    # recommendation: antecedent in basket -> r1 (conf 1.0, ->2), r3 (0.9, ->4), r2 (0.75, ->3), r4 (0.6, ->1)
    assert out["rec1"] == "2" and out["rec2"] == "4"
    assert out["conf"] == 1.0 and out["rid"] == "r1"
    # exclusive: consequent not in the basket -> r1 first
    assert out["excl"] == "2"
    # ruleAssociation: antecedent and consequent in the basket -> r2 (0.75) before r4 (0.6)
    assert out["assoc"] == "{1}->{3}"
    assert out["by_lift"] == "r2"  # lift 1.5
    assert out["low_support"] == 0.5  # ascending support: r2 / r3 tie at 0.5, document order


def test_no_matching_rule_is_missing(model):
    out = model.predict_with_outputs(DenseVector(2.0, 2.0, 2.0)).outputs  # basket {2}
    assert out["rec1"] is None and out["excl"] is None
    assert out["conf"] is None or math.isnan(out["conf"])


def test_exclusive_recommendation_drops_only_contained_consequents():
    """``exclusiveRecommendation`` drops a rule only when its whole consequent is already
    in the basket (PMML; parity unpinned — no JPMML here). A two-item consequent {1, 3} against
    the basket {2, 3} overlaps in one item and is still recommended."""
    doc = DOC.replace('<AssociationRule id="r1" support="1.0" confidence="1.0" lift="1.0" antecedent="1" consequent="2"/>',
                      '<AssociationRule id="r1" support="1.0" confidence="1.0" lift="1.0" antecedent="2" consequent="4"/>')
    m = PmmlModel.from_string(doc)
    out = m.predict_with_outputs(DenseVector(2.0, 3.0, float("nan"))).outputs  # basket {2, 3}
    assert out["excl"] == "{1,3}", out
    # and a fully contained consequent is excluded: basket {1, 2, 3} contains {1, 3}
    out = m.predict_with_outputs(DenseVector(1.0, 2.0, 3.0)).outputs
    assert out["excl"] == "4", out  # r1 excluded; r3 ({1,3} -> {4}) is next
