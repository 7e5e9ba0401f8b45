"""weightedConfidence / aggregateNodes sibling mixtures on the device path:
seeded random classification TreeModels and MiningModel ensembles of them (majority / weighted
majority vote, average / weighted average) through the GENERAL layout's numpy twin
(``runtime/general_tree.py::emulate_general`` = ``tree.hip::gen_walk`` + ``gen_mixture``) vs the
float64 oracle (``models/tree.py::_mixture``): validity equal, labels equal wherever the oracle's
winning class is not within fp32 of a tie, probabilities within fp32."""

import random

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml
from tests.test_native_walk import NF, _header, _inputs, _ms, _node

CATS = ["a", "b", "c"]


def mixture_doc(seed: int, n_trees: int = 1, method: str = "majorityVote") -> str:
    rng = random.Random(seed)
    strat = ["weightedConfidence", "aggregateNodes"][seed % 2]
    trees = []
    for t in range(n_trees):
        notrue = rng.choice(["returnNullPrediction", "returnLastPrediction"])
        root = _node(rng, rng.randrange(2, 5), [], True, "<True/>", consistent=True)
        trees.append(f'<TreeModel functionName="classification" missingValueStrategy="{strat}" '
                     f'noTrueChildStrategy="{notrue}">{_ms()}{root}</TreeModel>')
    tgt = '<DataField name="y" optype="categorical" dataType="string">' + \
        "".join(f'<Value value="{c}"/>' for c in CATS) + "</DataField>"
    if n_trees == 1:
        return _header(tgt) + trees[0] + "</PMML>"
    segs = "".join(f'<Segment id="s{i}" weight="{0.5 + i % 3}"><True/>{t}</Segment>' for i, t in enumerate(trees))
    return (_header(tgt) + f'<MiningModel functionName="classification">{_ms()}'
            f'<Segmentation multipleModelMethod="{method}">{segs}</Segmentation></MiningModel></PMML>')


def _check(doc: str, seed: int):
    from flink_jpmml_amd.runtime.general_tree import emulate_general, pack_general
    from flink_jpmml_amd.runtime.plans import TreePlan

    c = CompiledPmml.from_string(doc)
    spec = TreePlan._general_spec(c)
    packed = pack_general(spec.trees, spec.weights, spec.P, c.schema)
    assert packed["mix_mass"] is not None
    X = _inputs(seed, 800).astype(np.float32).astype(np.float64)
    acc = emulate_general(packed, X, spec.P, len(spec.trees))
    valid = ~np.isnan(acc).any(axis=1)
    res = c.result(X)
    assert (valid == res.valid).all(), (seed, int((valid != res.valid).sum()))
    if not valid.any():
        return
    probs = acc[valid] * spec.epi.get("a", 1.0)
    ref = np.nan_to_num(res.probs[valid])
    np.testing.assert_allclose(probs, ref, rtol=0, atol=5e-6)
    lab = np.argmax(np.nan_to_num(acc[valid]), axis=1)
    srt = np.sort(ref, axis=1)
    clear = srt[:, -1] - srt[:, -2] > 1e-5  # not within fp32 of a tie
    assert (lab[clear] == res.value[valid][clear]).all()


@pytest.mark.parametrize("seed", range(40))
def test_random_mixture_trees_match_oracle(seed):
    _check(mixture_doc(seed), seed)


@pytest.mark.parametrize("method", ["majorityVote", "weightedMajorityVote", "average", "weightedAverage"])
@pytest.mark.parametrize("seed", range(6))
def test_random_mixture_ensembles_match_oracle(seed, method):
    _check(mixture_doc(100 + seed, n_trees=5, method=method), seed)
