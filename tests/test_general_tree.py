"""GENERAL tree layout (predicate VM): random PMML TreeModels with multiway splits, compound
(and / or / xor / surrogate) and set predicates, every missing-value strategy and both
noTrueChild strategies. The numpy twin of the kernel walk must reproduce the float64 oracle
exactly (selected node per row); GPU parity is in test_gpu_kernels.py."""

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml

NS = "http://www.dmg.org/PMML-4_4"
CATS = "abcde"


class _Gen:
    def __init__(self, rng, depth, strategy):
        self.rng = rng
        self.depth = depth
        self.strategy = strategy
        self.nid = 0

    def simple(self):
        r = self.rng
        f = int(r.integers(4))
        op = r.choice(["lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual", "equal", "notEqual",
                       "isMissing", "isNotMissing"], p=[.22, .22, .17, .17, .06, .06, .05, .05])
        if op in ("isMissing", "isNotMissing"):
            return f'<SimplePredicate field="x{f}" operator="{op}"/>'
        v = float(np.round(r.normal(), 1)) if op not in ("equal", "notEqual") else float(r.integers(-1, 2))
        return f'<SimplePredicate field="x{f}" operator="{op}" value="{v}"/>'

    def setp(self):
        k = int(self.rng.integers(1, 4))
        vals = self.rng.choice(list(CATS), size=k, replace=False)
        op = self.rng.choice(["isIn", "isNotIn"])
        return (f'<SimpleSetPredicate field="c" booleanOperator="{op}"><Array type="string" n="{k}">'
                + " ".join(vals) + '</Array></SimpleSetPredicate>')

    def pred(self):
        u = self.rng.random()
        if u < 0.5:
            return self.simple()
        if u < 0.7:
            return self.setp()
        op = self.rng.choice(["and", "or", "xor", "surrogate"])
        parts = [self.simple() if self.rng.random() < 0.7 else self.setp() for _ in range(int(self.rng.integers(2, 4)))]
        if op == "surrogate" and self.rng.random() < 0.5:
            parts.append("<True/>")
        return f'<CompoundPredicate booleanOperator="{op}">' + "".join(parts) + "</CompoundPredicate>"

    def node(self, pred, d):
        self.nid += 1
        my = self.nid
        score = f'{self.rng.normal():.3f}'
        if d >= self.depth or self.rng.random() < 0.15:
            return f'<Node id="n{my}" score="{score}">{pred}</Node>'
        nc = int(self.rng.integers(2, 5))
        kids = [self.node(self.pred() if (i < nc - 1 or self.rng.random() < 0.6) else "<True/>", d + 1)
                for i in range(nc)]
        dflt = f' defaultChild="n{my + 1}"' if self.strategy == "defaultChild" else ""
        return f'<Node id="n{my}" score="{score}"{dflt}>{pred}' + "".join(kids) + "</Node>"


def general_tree_doc(seed, strategy="none", no_true="returnNullPrediction", n_trees=1, classification=False):
    rng = np.random.default_rng(seed)
    dd = "".join(f'<DataField name="x{j}" optype="continuous" dataType="double"/>' for j in range(4))
    dd += '<DataField name="c" optype="categorical" dataType="string">' + "".join(
        f'<Value value="{v}"/>' for v in CATS) + "</DataField>"
    if classification:
        dd += '<DataField name="y" optype="categorical" dataType="string"><Value value="0"/><Value value="1"/>' \
              '<Value value="2"/></DataField>'
    else:
        dd += '<DataField name="y" optype="continuous" dataType="double"/>'
    ms = '<MiningSchema><MiningField name="y" usageType="target"/>' + "".join(
        f'<MiningField name="x{j}"/>' for j in range(4)) + '<MiningField name="c"/></MiningSchema>'
    fn = "classification" if classification else "regression"

    def tree():
        g = _Gen(rng, 4, strategy)
        body = g.node("<True/>", 0)
        if classification:  # scores -> class labels
            import re

            body = re.sub(r'score="[-0-9.]+"', lambda m: f'score="{rng.choice(list("012"))}"', body)
        return (f'<TreeModel functionName="{fn}" missingValueStrategy="{strategy}" '
                f'noTrueChildStrategy="{no_true}">{ms}{body}</TreeModel>')

    if n_trees == 1:
        model = tree()
    else:
        method = "majorityVote" if classification else "average"
        model = (f'<MiningModel functionName="{fn}">{ms}<Segmentation multipleModelMethod="{method}">'
                 + "".join(f'<Segment id="{i}"><True/>{tree()}</Segment>' for i in range(n_trees))
                 + "</Segmentation></MiningModel>")
    return f'<PMML version="4.4" xmlns="{NS}"><DataDictionary>{dd}</DataDictionary>{model}</PMML>'


def general_inputs(n, seed):
    rng = np.random.default_rng(seed)
    X = np.empty((n, 5))
    X[:, :4] = np.round(rng.normal(size=(n, 4)), 1)  # hits the split constants exactly
    X[:, 4] = rng.integers(0, len(CATS), n)
    X[rng.random((n, 5)) < 0.08] = np.nan
    return X.astype(np.float32).astype(np.float64)  # the engine's inputs are fp32 records


CASES = [(s, nt) for s in ("none", "lastPrediction", "nullPrediction", "defaultChild")
         for nt in ("returnNullPrediction", "returnLastPrediction")]


@pytest.mark.parametrize("strategy,no_true", CASES)
def test_general_layout_emulation_matches_oracle(strategy, no_true):
    from flink_jpmml_amd.runtime.general_tree import emulate_general, pack_general
    from flink_jpmml_amd.runtime.plans import TreePlan

    from test_lowering import _scores

    for seed in range(3):
        c = CompiledPmml.from_string(general_tree_doc(seed, strategy, no_true))
        spec = TreePlan._general_spec(c)
        packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
        X = general_inputs(600, seed)
        acc = emulate_general(packed, X, spec.P, len(spec.trees))
        ref, vref = c.score_matrix_oracle(X)
        out = _scores(spec, acc)
        assert (np.isfinite(out) == vref).all(), (seed, strategy, no_true)
        np.testing.assert_allclose(out[vref], ref[vref], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("classification", [False, True])
def test_general_layout_ensembles(classification):
    from flink_jpmml_amd.runtime.general_tree import emulate_general, pack_general
    from flink_jpmml_amd.runtime.plans import TreePlan

    from test_lowering import _scores

    c = CompiledPmml.from_string(general_tree_doc(11, "defaultChild", "returnLastPrediction", n_trees=7,
                                                  classification=classification))
    spec = TreePlan._general_spec(c)
    packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
    X = general_inputs(500, 4)
    acc = emulate_general(packed, X, spec.P, len(spec.trees))
    ref, vref = c.score_matrix_oracle(X)
    out = _scores(spec, acc)
    assert (np.isfinite(out) == vref).all()
    np.testing.assert_allclose(out[vref], ref[vref], rtol=1e-6, atol=1e-6)
