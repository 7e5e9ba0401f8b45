"""Derived fields (TransformationDictionary / LocalTransformations): the lowering to the derive
kernel's postfix program is checked on the CPU against the float64 oracle through the program's
numpy twin (``runtime.derive.emulate``), and the field-layout decisions (alias vs program) are
pinned. GPU parity of the kernel itself lives in ``test_gpu_kernels.py``.

Tolerance: derived columns are stored as fp32 (what every model kernel consumes), so they are
compared with the oracle's fp64 values rounded to fp32 (rtol 1e-6 covers fp64 libm differences)."""

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.derive import emulate, plan_field_layout, referenced_fields

NS = "http://www.dmg.org/PMML-4_4"

DICT = """
 <DataDictionary>
  <DataField name="a" optype="continuous" dataType="double"/>
  <DataField name="b" optype="continuous" dataType="double"/>
  <DataField name="c" optype="categorical" dataType="string"><Value value="red"/><Value value="green"/><Value value="blue"/></DataField>
  <DataField name="y" optype="continuous" dataType="double"/>
 </DataDictionary>
 <TransformationDictionary>
  <DerivedField name="log_a" optype="continuous" dataType="double"><Apply function="ln"><FieldRef field="a"/></Apply></DerivedField>
  <DerivedField name="ab" optype="continuous" dataType="double"><Apply function="+" mapMissingTo="-1"><Apply function="*"><FieldRef field="a"/><Constant>2.5</Constant></Apply><FieldRef field="b"/></Apply></DerivedField>
  <DerivedField name="nb" optype="continuous" dataType="double"><NormContinuous field="b" outliers="asExtremeValues" mapMissingTo="0"><LinearNorm orig="-2" norm="0"/><LinearNorm orig="0" norm="0.5"/><LinearNorm orig="3" norm="1"/></NormContinuous></DerivedField>
  <DerivedField name="is_red" optype="continuous" dataType="double"><NormDiscrete field="c" value="red" mapMissingTo="-1"/></DerivedField>
  <DerivedField name="bin_a" optype="continuous" dataType="integer"><Discretize field="a" mapMissingTo="9" defaultValue="7"><DiscretizeBin binValue="1"><Interval closure="openClosed" rightMargin="0"/></DiscretizeBin><DiscretizeBin binValue="2"><Interval closure="openOpen" leftMargin="0" rightMargin="1.5"/></DiscretizeBin></Discretize></DerivedField>
  <DerivedField name="code_c" optype="continuous" dataType="double"><MapValues outputColumn="out" defaultValue="0" mapMissingTo="-5"><FieldColumnPair field="c" column="col"/><InlineTable><row><col>red</col><out>10</out></row><row><col>blue</col><out>30</out></row></InlineTable></MapValues></DerivedField>
  <DerivedField name="mx" optype="continuous" dataType="double"><Apply function="max"><FieldRef field="a"/><FieldRef field="b"/><Constant>0.25</Constant></Apply></DerivedField>
  <DerivedField name="md" optype="continuous" dataType="double"><Apply function="median"><FieldRef field="a"/><FieldRef field="b"/><Constant>0.1</Constant><FieldRef field="ab"/></Apply></DerivedField>
  <DerivedField name="cond" optype="continuous" dataType="double"><Apply function="if"><Apply function="greaterThan"><FieldRef field="ab"/><Constant>1</Constant></Apply><Apply function="sqrt" defaultValue="-3"><FieldRef field="b"/></Apply><Constant>-2</Constant></Apply></DerivedField>
  <DerivedField name="miss_b" optype="continuous" dataType="double"><Apply function="isMissing"><FieldRef field="b"/></Apply></DerivedField>
  <DerivedField name="modv" optype="continuous" dataType="double"><Apply function="modulo"><FieldRef field="ab"/><Constant>-0.75</Constant></Apply></DerivedField>
  <DerivedField name="fa" optype="continuous" dataType="float"><FieldRef field="a"/></DerivedField>
  <DerivedField name="in_c" optype="continuous" dataType="double"><Apply function="isIn"><FieldRef field="c"/><Constant>red</Constant><Constant>blue</Constant></Apply></DerivedField>
  <DerivedField name="notin_a" optype="continuous" dataType="double"><Apply function="isNotIn" mapMissingTo="5"><FieldRef field="a"/><Constant>0</Constant><Constant>1.5</Constant></Apply></DerivedField>
  <DerivedField name="erf_b" optype="continuous" dataType="double"><Apply function="erf"><FieldRef field="b"/></Apply></DerivedField>
  <DerivedField name="ncdf_a" optype="continuous" dataType="double"><Apply function="stdNormalCDF"><FieldRef field="a"/></Apply></DerivedField>
  <DerivedField name="npdf_b" optype="continuous" dataType="double"><Apply function="stdNormalPDF"><FieldRef field="b"/></Apply></DerivedField>
  <DerivedField name="nidf_a" optype="continuous" dataType="double"><Apply function="stdNormalIDF"><Apply function="/"><Apply function="+"><FieldRef field="a"/><Constant>2.01</Constant></Apply><Constant>5.1</Constant></Apply></Apply></DerivedField>
  <DerivedField name="hyp" optype="continuous" dataType="double"><Apply function="hypot"><FieldRef field="a"/><FieldRef field="b"/></Apply></DerivedField>
  <DerivedField name="at2" optype="continuous" dataType="double"><Apply function="atan2"><FieldRef field="b"/><FieldRef field="a"/></Apply></DerivedField>
 </TransformationDictionary>
"""

DERIVED = ["log_a", "ab", "nb", "is_red", "bin_a", "code_c", "mx", "md", "cond", "miss_b", "modv", "fa", "in_c",
           "notin_a", "erf_b", "ncdf_a", "npdf_b", "nidf_a", "hyp", "at2"]  # last six: PMML 4.4 functions


def regression_doc() -> str:
    preds = "".join(f'<NumericPredictor name="{n}" coefficient="{0.1 * (i + 1):.1f}"/>' for i, n in enumerate(DERIVED))
    return (f'<PMML version="4.4" xmlns="{NS}">{DICT}'
            ' <RegressionModel functionName="regression">'
            '  <MiningSchema><MiningField name="y" usageType="target"/><MiningField name="a"/>'
            '<MiningField name="b"/><MiningField name="c"/></MiningSchema>'
            f'  <RegressionTable intercept="0.5">{preds}</RegressionTable>'
            ' </RegressionModel></PMML>')


def tree_doc() -> str:
    return (f'<PMML version="4.4" xmlns="{NS}">{DICT}'
            ' <TreeModel functionName="regression" missingValueStrategy="defaultChild" splitCharacteristic="binarySplit">'
            '  <MiningSchema><MiningField name="y" usageType="target"/><MiningField name="a"/>'
            '<MiningField name="b"/><MiningField name="c"/></MiningSchema>'
            '  <Node id="0" defaultChild="1"><True/>'
            '   <Node id="1" defaultChild="3"><SimplePredicate field="ab" operator="lessThan" value="0.7"/>'
            '    <Node id="3" score="-1.5"><SimplePredicate field="nb" operator="lessOrEqual" value="0.4"/></Node>'
            '    <Node id="4" score="2.25"><SimplePredicate field="nb" operator="greaterThan" value="0.4"/></Node>'
            '   </Node>'
            '   <Node id="2" defaultChild="5"><SimplePredicate field="ab" operator="greaterOrEqual" value="0.7"/>'
            '    <Node id="5" score="0.125"><SimplePredicate field="code_c" operator="lessThan" value="20"/></Node>'
            '    <Node id="6" score="4.5"><SimplePredicate field="code_c" operator="greaterOrEqual" value="20"/></Node>'
            '   </Node>'
            '  </Node>'
            ' </TreeModel></PMML>')


def inputs(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    X = np.empty((n, 3))
    X[:, 0] = rng.uniform(-2, 3, n)
    X[:, 1] = rng.normal(0, 2, n)
    X[:, 2] = rng.integers(0, 3, n)
    X[rng.random((n, 3)) < 0.1] = np.nan
    X[:8, 0] = [0.0, 1.5, -1e-30, 1.5000001, 0.0, np.nan, 2.0, -0.0]  # Discretize bin edges
    return X.astype(np.float32).astype(np.float64)


def test_referenced_fields_walks_model_elements():
    c = CompiledPmml.from_string(tree_doc())
    assert referenced_fields(c.model) == ["ab", "nb", "code_c"]
    c2 = CompiledPmml.from_string(regression_doc())
    assert referenced_fields(c2.model) == DERIVED


def test_program_matches_oracle_columns():
    c = CompiledPmml.from_string(regression_doc())
    layout = plan_field_layout(c)
    prog = layout.program
    assert prog is not None and layout.columns == DERIVED
    assert prog.max_stack <= 16
    X = inputs()
    P, ok = c.prepare(X)
    assert ok.all()
    got = emulate(prog, P)
    cols = c.columns(P)
    for j, name in enumerate(prog.selected):
        ref = cols.get(name).astype(np.float32)
        # fields fed by the double field `ab` see it rounded to fp32 (see runtime/derive.py): atol
        np.testing.assert_allclose(got[:, j], ref, rtol=1e-6, atol=2e-6, equal_nan=True, err_msg=name)


def test_program_regression_score_matches_oracle():
    c = CompiledPmml.from_string(regression_doc())
    prog = plan_field_layout(c).program
    X = inputs(seed=3)
    P, _ = c.prepare(X)
    D = emulate(prog, P).astype(np.float64)
    coef = np.array([0.1 * (i + 1) for i in range(len(DERIVED))])
    s = D @ coef + 0.5
    ref, vref = c.score_matrix_oracle(X)
    assert (np.isfinite(s) == vref).all()  # ln(0) = -inf: no prediction
    np.testing.assert_allclose(s[vref], ref[vref], rtol=1e-5, atol=1e-5)


def test_tree_on_derived_fields_uses_program():
    c = CompiledPmml.from_string(tree_doc())
    layout = plan_field_layout(c, allow_alias=True)
    assert layout.program is not None
    assert layout.columns == ["ab", "nb", "code_c"]
    assert layout.program.derived == ["ab", "nb", "code_c"]


def test_float_cast_aliases_need_no_program():
    from flink_jpmml_amd.bench.synth import gbdt_pmml

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=4, depth=3, n_features=5, seed=2, float_casts=True))
    layout = plan_field_layout(c, allow_alias=True)
    assert layout.program is None
    assert layout.field_index["float(f3)"] == layout.field_index["f3"] == 3
    # without aliasing (non-tree plans) the same casts become a program
    assert plan_field_layout(c, allow_alias=False).program is not None


def test_float_cast_gbdt_lowering_matches_oracle():
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.runtime.derive import FieldView

    from test_lowering import _scores, emulate_perfect

    c = CompiledPmml.from_string(gbdt_pmml(n_trees=20, depth=4, n_features=6, seed=5, float_casts=True))
    view = FieldView(c, plan_field_layout(c), prepared=False)
    X = stream_matrix(500, 6, seed=1, missing_rate=0.05)
    ref, vref = c.score_matrix_oracle(X)
    spec, acc = emulate_perfect(view, X)
    assert len(spec.trees) == 20
    assert np.max(np.abs(_scores(spec, acc)[vref] - ref[vref])) < 1e-5


@pytest.mark.parametrize("bad", ['<Apply function="uppercase"><FieldRef field="c"/></Apply>',
                                 '<Apply function="+"><FieldRef field="a"/></Apply>'])
def test_unsupported_expressions_stay_on_host(bad):
    from flink_jpmml_amd.runtime.plans import NotLowerable

    doc = regression_doc().replace('<Apply function="ln"><FieldRef field="a"/></Apply>', bad)
    c = CompiledPmml.from_string(doc)
    with pytest.raises(NotLowerable):
        plan_field_layout(c)


def categorical_tree_doc(strategy: str = "defaultChild") -> str:
    """LightGBM / R style categorical splits: isIn / isNotIn sets and == / != on a string field."""
    return (f'<PMML version="4.4" xmlns="{NS}"><DataDictionary>'
            '<DataField name="x" optype="continuous" dataType="double"/>'
            '<DataField name="cat" optype="categorical" dataType="string">'
            + "".join(f'<Value value="{v}"/>' for v in "abcdef") +
            '</DataField><DataField name="y" optype="continuous" dataType="double"/></DataDictionary>'
            f'<TreeModel functionName="regression" missingValueStrategy="{strategy}" splitCharacteristic="binarySplit">'
            '<MiningSchema><MiningField name="y" usageType="target"/><MiningField name="x"/><MiningField name="cat"/>'
            '</MiningSchema>'
            '<Node id="0" defaultChild="2"><True/>'
            ' <Node id="1" defaultChild="3"><SimpleSetPredicate field="cat" booleanOperator="isIn">'
            '<Array type="string" n="3">a c "e"</Array></SimpleSetPredicate>'
            '  <Node id="3" score="1.0"><SimplePredicate field="x" operator="lessThan" value="0.25"/></Node>'
            '  <Node id="4" defaultChild="5"><SimplePredicate field="x" operator="greaterOrEqual" value="0.25"/>'
            '   <Node id="5" score="2.0"><SimplePredicate field="cat" operator="equal" value="a"/></Node>'
            '   <Node id="6" score="3.0"><SimplePredicate field="cat" operator="notEqual" value="a"/></Node>'
            '  </Node>'
            ' </Node>'
            ' <Node id="2" defaultChild="7"><SimpleSetPredicate field="cat" booleanOperator="isNotIn">'
            '<Array type="string" n="3">a c "e"</Array></SimpleSetPredicate>'
            '  <Node id="7" score="4.0"><SimpleSetPredicate field="cat" booleanOperator="isNotIn">'
            '<Array type="string" n="1">f</Array></SimpleSetPredicate></Node>'
            '  <Node id="8" score="5.0"><SimpleSetPredicate field="cat" booleanOperator="isIn">'
            '<Array type="string" n="1">f</Array></SimpleSetPredicate></Node>'
            ' </Node>'
            '</Node></TreeModel></PMML>')


def cat_inputs(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    X = np.stack([rng.normal(0, 1, n), rng.integers(0, 6, n).astype(float)], axis=1)
    X[rng.random((n, 2)) < 0.08] = np.nan
    return X


@pytest.mark.parametrize("strategy", ["defaultChild", "nullPrediction"])
def test_categorical_splits_lower_to_membership_columns(strategy):
    from flink_jpmml_amd.runtime.derive import FieldView

    from test_lowering import _scores, emulate_perfect

    c = CompiledPmml.from_string(categorical_tree_doc(strategy))
    layout = plan_field_layout(c)
    prog = layout.program
    members = [n for n in layout.columns if n.startswith("__in__(")]
    assert sorted(members) == ["__in__(cat|a)", "__in__(cat|a|c|e)", "__in__(cat|f)"]
    X = cat_inputs()
    P, ok = c.prepare(X)
    Xd = emulate(prog, P)
    view = FieldView(c, layout, prepared=True)
    spec, acc = emulate_perfect(view, Xd)
    ref, vref = c.score_matrix_oracle(X)
    out = _scores(spec, acc)
    assert (np.isfinite(out) == vref).all()
    assert (out[vref] == ref[vref]).all()
