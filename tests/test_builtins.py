"""PMML built-in functions of JPMML-Evaluator's function library beyond arithmetic: isIn /
isNotIn, matches and the string functions (uppercase, lowercase, substring, trimBlanks, concat,
replace, formatNumber), evaluated by the float64 oracle (string results re-encoded into the
derived field's vocabulary)."""

import numpy as np

from flink_jpmml_amd.runtime.compiled import CompiledPmml

DOC = """<?xml version="1.0"?>
<PMML version="4.3" xmlns="http://www.dmg.org/PMML-4_3">
 <Header/>
 <DataDictionary>
  <DataField name="color" optype="categorical" dataType="string">
   <Value value=" Red"/><Value value="green "/><Value value="BLUE"/></DataField>
  <DataField name="x" optype="continuous" dataType="double"/>
  <DataField name="y" optype="continuous" dataType="double"/>
 </DataDictionary>
 <TransformationDictionary>
  <DerivedField name="clean" optype="categorical" dataType="string">
   <Apply function="lowercase"><Apply function="trimBlanks"><FieldRef field="color"/></Apply></Apply>
  </DerivedField>
  <DerivedField name="is_warm" optype="continuous" dataType="double">
   <Apply function="isIn"><FieldRef field="clean"/><Constant>red</Constant><Constant>orange</Constant></Apply>
  </DerivedField>
  <DerivedField name="not_small" optype="continuous" dataType="double">
   <Apply function="isNotIn"><FieldRef field="x"/><Constant>1</Constant><Constant>2</Constant></Apply>
  </DerivedField>
  <DerivedField name="tag" optype="categorical" dataType="string">
   <Apply function="concat"><Apply function="uppercase"><Apply function="substring"><FieldRef field="clean"/>
    <Constant>1</Constant><Constant>2</Constant></Apply></Apply><Constant>-</Constant>
    <Apply function="formatNumber"><FieldRef field="x"/><Constant>%03d</Constant></Apply></Apply>
  </DerivedField>
  <DerivedField name="has_e" optype="continuous" dataType="double">
   <Apply function="matches"><FieldRef field="clean"/><Constant>e+n</Constant></Apply>
  </DerivedField>
  <DerivedField name="swapped" optype="categorical" dataType="string">
   <Apply function="replace"><FieldRef field="clean"/><Constant>(r)(e)</Constant><Constant>$2$1</Constant></Apply>
  </DerivedField>
  <DerivedField name="tagged_blue" optype="continuous" dataType="double">
   <Apply function="isIn"><FieldRef field="swapped"/><Constant>erd</Constant></Apply>
  </DerivedField>
 </TransformationDictionary>
 <RegressionModel functionName="regression">
  <MiningSchema><MiningField name="color"/><MiningField name="x"/><MiningField name="y" usageType="target"/></MiningSchema>
  <Output>
   <OutputField name="out_tag" feature="transformedValue" dataType="string"><FieldRef field="tag"/></OutputField>
   <OutputField name="out_swapped" feature="transformedValue" dataType="string"><FieldRef field="swapped"/></OutputField>
  </Output>
  <RegressionTable intercept="0.0">
   <NumericPredictor name="is_warm" coefficient="100"/>
   <NumericPredictor name="not_small" coefficient="10"/>
   <NumericPredictor name="has_e" coefficient="1"/>
   <NumericPredictor name="tagged_blue" coefficient="1000"/>
  </RegressionTable>
 </RegressionModel>
</PMML>"""


def test_string_builtins_and_membership():
    from flink_jpmml_amd import DenseVector, PmmlModel

    m = PmmlModel.from_string(DOC)
    c = m.evaluator.model
    colors = c.schema.values["color"]
    X = np.array([[colors.index(" Red"), 7.0], [colors.index("green "), 1.0], [colors.index("BLUE"), 12.0]])
    s, v = c.score_matrix_oracle(X)
    # red: warm 100 + not_small 10 + has_e 1 ("red" matches e+n? no: "e" then "d") -> 110; swapped "erd" -> +1000
    assert v.all()
    np.testing.assert_array_equal(s, [1110.0, 1.0, 10.0])  # green: "een" matches e+n -> 1; x=1 is small
    _, outs = c.evaluate_prepared(c.prepare(X)[0])
    tags = [c.schema.decode("out_tag", v) for v in outs["out_tag"]]
    swapped = [c.schema.decode("out_swapped", v) for v in outs["out_swapped"]]
    assert tags == ["RE-007", "GR-001", "BL-012"]
    assert swapped == ["erd", "geren", "blue"]
    # the per-record API rejects a number for a string field, as the reference's JPMML prepare does
    assert m.predict(DenseVector(0.0, 7.0)).value.is_empty
