"""GPU twin of test_predicate_fuzz.py / test_literal_fuzz.py.

* Segment predicates past the fused VM's 32-entry stack fall back to the tensor-op predicates and
  still score like the float64 oracle; predicates at the limit run through ``segment.hip``'s
  ``seg_predicate`` and score like the oracle.
* Seeded random nested predicates (And / Or / Xor / Surrogate, missing inputs) in whole segmented
  documents: device plan vs oracle.
* Literal mutants the loader accepts (numbers swapped for numbers) score on the device plans like
  the oracle; the junk ones never reach a plan (rejected at load).
"""

import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _score(gpu, txt, n=20_000, seed=4, missing=0.1):
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **ScoringConfig(device=gpu, fallback="error").lowering_opts())
    X = stream_matrix(n, c.n_features, seed=seed, missing_rate=missing)
    s, v = plan.score(X)
    s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    np.testing.assert_allclose(s[v], ref[v], rtol=1e-5, atol=1e-5)
    return plan, v


def test_deep_segment_predicates_on_gpu(gpu):
    from test_predicate_fuzz import segmented_with_predicates

    from flink_jpmml_amd.pmml import ir

    deep = ir.CompoundPredicate("and", [ir.SimplePredicate("f0", "greaterThan", "-1.5")] * 20 +
                                [ir.CompoundPredicate("and", [ir.SimplePredicate("f1", "lessThan", "1.5")] * 20)])
    at_limit = ir.CompoundPredicate("or", [ir.SimplePredicate(f"f{i % 6}", "greaterThan", "1.2")
                                           for i in range(32)])
    for p, fused in ((deep, False), (at_limit, True)):
        plan, v = _score(gpu, segmented_with_predicates([p, p]))
        assert v.any()
        assert (getattr(plan, "inner", plan)._red is not None) == fused


@pytest.mark.parametrize("seed", range(3))
def test_random_nested_segment_predicates_on_gpu(gpu, seed):
    from test_predicate_fuzz import random_predicate, segmented_with_predicates

    rng = random.Random(1000 + seed)
    for method in ("selectFirst", "max", "average"):
        preds = [random_predicate(rng, rng.randrange(2, 7)) for _ in range(3)]
        _score(gpu, segmented_with_predicates(preds, method=method, seed=seed), n=8192)


def test_accepted_literal_mutants_on_gpu(gpu, monkeypatch):
    from test_literal_fuzz import JUNK, NUMBERS, documents, sites

    from flink_jpmml_amd.api.exceptions import PmmlParseError
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rng = random.Random("gpu-literals")
    scored = rejected = 0
    for name in ("gbdt", "segmented", "prefixed"):
        text = documents()[name]
        where = [w for w in sites(text) if w[0] != "n"]
        for _ in range(6):
            kind, fld, a, b = rng.choice(where)
            lit = rng.choice(NUMBERS + JUNK[:3])
            mutated = text[:a] + lit + text[b:]
            try:
                CompiledPmml.from_string(mutated)
            except PmmlParseError:
                rejected += 1
                continue
            _score(gpu, mutated, n=4096)
            scored += 1
    assert scored > 5 and rejected > 0
