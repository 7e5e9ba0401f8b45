"""weightedConfidence / aggregateNodes on the MI355X (``tree.hip::gen_mixture``) vs the float64
oracle, with ``fallback="error"`` semantics: the plan must lower."""

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml
from tests._suite import gpu_seeds
from tests.test_mixture_lowering import mixture_doc
from tests.test_native_walk import _inputs

pytestmark = pytest.mark.gpu


def _numeric_labels(doc: str) -> str:
    """Categories 1 / 2 / 3 instead of a / b / c: a prediction is a Score only when its label
    parses as a number (the reference's extract_target), so the valid masks compare row by row."""
    for k, v in (("a", "1"), ("b", "2"), ("c", "3")):
        doc = doc.replace(f'value="{k}"', f'value="{v}"').replace(f'score="{k}"', f'score="{v}"')
    return doc


def _run(gpu, doc, seed):
    doc = _numeric_labels(doc)
    c = CompiledPmml.from_string(doc)
    plan = c.plan(gpu)
    inner = getattr(plan, "inner", plan)  # set / equality splits add a membership derive pass
    assert inner.layout == "general" and inner.mix_mass is not None
    X = _inputs(seed, 20000)
    s, v = plan.score(X)
    v = v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), int((v != vref).sum())
    s = s.cpu().numpy()
    assert (s[v] == ref[v]).mean() >= 0.999  # labels (ties within fp32 may flip)
    res = c.result(X)
    assert (res.valid == vref).all()
    # labels: score is the label's table value (categories a/b/c are not numbers -> compare via probs)
    import torch

    probs = torch.empty((len(X), inner.C), dtype=torch.float32, device=gpu)
    s2 = torch.empty(len(X), dtype=torch.float32, device=gpu)
    v2 = torch.empty(len(X), dtype=torch.uint8, device=gpu)
    Xd = torch.as_tensor(X.astype(np.float32), device=gpu)
    plan.launch(Xd, s2, v2, probs=probs)
    torch.cuda.synchronize()
    p = probs.cpu().numpy()[v]
    pref = np.nan_to_num(res.probs[v])
    np.testing.assert_allclose(p, pref, rtol=0, atol=2e-5)


@pytest.mark.parametrize("seed", gpu_seeds(24, 8))
def test_mixture_trees_on_gpu(gpu, seed):
    _run(gpu, mixture_doc(seed), seed)


@pytest.mark.parametrize("method", ["majorityVote", "weightedMajorityVote", "average", "weightedAverage"])
def test_mixture_ensembles_on_gpu(gpu, method):
    _run(gpu, mixture_doc(200, n_trees=9, method=method), 3)
