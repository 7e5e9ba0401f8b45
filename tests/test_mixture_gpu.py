"""weightedConfidence / aggregateNodes on the MI355X (``tree.hip::gen_mixture``) vs the float64
oracle, with ``fallback="error"`` semantics: the plan must lower."""

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml
from tests._suite import gpu_seeds
from tests.test_mixture_lowering import mixture_doc
from tests.test_native_walk import _inputs

pytestmark = pytest.mark.gpu


def _run(gpu, doc, seed):
    c = CompiledPmml.from_string(doc)
    plan = c.plan(gpu)
    assert plan.layout == "general" and plan.mix_mass is not None
    X = _inputs(seed, 20000)
    s, v = plan.score(X)
    v = v.cpu().numpy().astype(bool)
    res = c.result(X)
    assert (v == res.valid).all(), int((v != res.valid).sum())
    # labels: score is the label's table value (categories a/b/c are not numbers -> compare via probs)
    import torch

    probs = torch.empty((len(X), plan.C), dtype=torch.float32, device=gpu)
    s2 = torch.empty(len(X), dtype=torch.float32, device=gpu)
    v2 = torch.empty(len(X), dtype=torch.uint8, device=gpu)
    Xd = torch.as_tensor(X.astype(np.float32), device=gpu)
    plan.launch(Xd, s2, v2, probs=probs)
    torch.cuda.synchronize()
    p = probs.cpu().numpy()[v]
    ref = np.nan_to_num(res.probs[v])
    np.testing.assert_allclose(p, ref, rtol=0, atol=2e-5)


@pytest.mark.parametrize("seed", gpu_seeds(24, 8))
def test_mixture_trees_on_gpu(gpu, seed):
    _run(gpu, mixture_doc(seed), seed)


@pytest.mark.parametrize("method", ["majorityVote", "weightedMajorityVote", "average", "weightedAverage"])
def test_mixture_ensembles_on_gpu(gpu, method):
    _run(gpu, mixture_doc(200, n_trees=9, method=method), 3)
