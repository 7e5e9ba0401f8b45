"""Segment predicate VM vs the oracle's three-valued logic.

``ops/csrc/segment.hip::seg_predicate`` evaluates a segment predicate as a postfix program whose
stack holds 2-bit TRUE / FALSE / UNKNOWN entries in ONE ``uint64``: a program that ever needs more
than 32 live entries would shift the oldest ones out and silently mis-select segments.
``runtime/segmented.py::predicate_programs`` therefore tracks the running postfix depth and refuses
(``NotLowerable`` → the tensor-op predicate path) anything deeper than ``SEG_STACK``.

Here a line-for-line model of the kernel — including the 64-bit shift register, so an overflow
WOULD show — runs seeded random nested And / Or / Xor / Surrogate trees (widths up to 32, depth up
to 8, Simple / SimpleSet / isMissing / True / False leaves, missing inputs) and must equal
``pmml/fields.py::eval_predicate`` on every row whenever ``predicate_programs`` accepts the program.
The GPU twin (``test_gpu_predicates.py``) runs deep predicates through the real kernel.
"""

from __future__ import annotations

import random

import numpy as np
import pytest

from flink_jpmml_amd.pmml import ir
from flink_jpmml_amd.pmml.fields import Columns, eval_predicate
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import NotLowerable
from flink_jpmml_amd.runtime.segmented import SEG_STACK, compile_predicate, predicate_programs

N_FIELDS = 4
M64 = (1 << 64) - 1
SV_F, SV_T, SV_U = 0, 1, 2


def _doc() -> CompiledPmml:
    """Any model over f0..f3 (only its schema / field order is used)."""
    fields = "".join(f'<DataField name="f{j}" optype="continuous" dataType="double"/>' for j in range(N_FIELDS))
    ms = '<MiningSchema><MiningField name="y" usageType="target"/>' + \
        "".join(f'<MiningField name="f{j}"/>' for j in range(N_FIELDS)) + "</MiningSchema>"
    return CompiledPmml.from_string(
        '<PMML xmlns="http://www.dmg.org/PMML-4_4" version="4.4"><DataDictionary>'
        f'{fields}<DataField name="y" optype="continuous" dataType="double"/></DataDictionary>'
        f'<RegressionModel functionName="regression">{ms}<RegressionTable intercept="0"/></RegressionModel></PMML>')


VALUES = [-1.0, -0.5, 0.0, 0.25, 0.5, 1.0]


def random_predicate(rng: random.Random, depth: int, max_width: int = 32) -> ir.Predicate:
    if depth == 0 or rng.random() < 0.3:
        k = rng.randrange(6)
        f = f"f{rng.randrange(N_FIELDS)}"
        if k == 0:
            return ir.TruePredicate()
        if k == 1:
            return ir.FalsePredicate()
        if k == 2:
            return ir.SimplePredicate(f, rng.choice(["isMissing", "isNotMissing"]))
        if k == 3:
            return ir.SimpleSetPredicate(f, rng.choice(["isIn", "isNotIn"]),
                                         [repr(v) for v in rng.sample(VALUES, rng.randrange(1, 4))])
        op = rng.choice(["equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual"])
        return ir.SimplePredicate(f, op, repr(rng.choice(VALUES)))
    width = rng.randrange(1, max_width + 1) if rng.random() < 0.2 else rng.randrange(1, 6)
    if depth > 3:  # keep the tree small: deep levels stay narrow (depth x width, not width^depth)
        width = min(width, 3)
    return ir.CompoundPredicate(rng.choice(["and", "or", "xor", "surrogate"]),
                                [random_predicate(rng, depth - 1, max_width) for _ in range(width)])


def postfix_depth(p: ir.Predicate) -> int:
    """Maximum live entries of the postfix evaluation of ``p`` (children pushed left to right)."""
    if not isinstance(p, ir.CompoundPredicate):
        return 1
    best = 0
    for i, q in enumerate(p.predicates):
        best = max(best, i + postfix_depth(q))
    return best


def kernel_model(insns, pool, pc: int, x: np.ndarray) -> int:
    """``seg_predicate`` line for line: 2-bit entries in a uint64 shift register."""
    st = 0
    while True:
        op_word, a, b, c = (int(v) for v in insns[pc])
        pc += 1
        op, arg = op_word & 0xFF, op_word >> 8
        if op == 0:
            return st & 3
        if op >= 7:
            any_t = any_f = any_u = False
            par, sur = 0, SV_U
            for _ in range(a):
                e = st & 3
                st >>= 2
                any_t |= e == SV_T
                any_f |= e == SV_F
                any_u |= e == SV_U
                par ^= 1 if e == SV_T else 0
                if e != SV_U:
                    sur = e
            if op == 7:
                v = SV_F if any_f else (SV_U if any_u else SV_T)
            elif op == 8:
                v = SV_T if any_t else (SV_U if any_u else SV_F)
            elif op == 9:
                v = SV_U if any_u else par
            else:
                v = sur
        elif op == 1:
            v = SV_T
        elif op == 2:
            v = SV_F
        else:
            xv = float(x[a])
            miss = xv != xv
            if op == 4:
                v = SV_T if miss else SV_F
            elif op == 5:
                v = SV_F if miss else SV_T
            elif miss:
                v = SV_U
            elif op == 3:
                t = pool[b]
                r = [xv == t, xv != t, xv < t, xv <= t, xv > t, xv >= t][arg]
                v = SV_T if r else SV_F
            else:
                inside = any(pool[b + i] == xv for i in range(c))
                v = SV_T if inside == (arg != 0) else SV_F
        st = ((st << 2) | v) & M64


def _inputs(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    X = rng.choice(np.array(VALUES + [0.75, -0.25]), size=(n, N_FIELDS))
    X[rng.random((n, N_FIELDS)) < 0.2] = np.nan
    return X.astype(np.float32).astype(np.float64)


def _oracle(c: CompiledPmml, p: ir.Predicate, X: np.ndarray) -> np.ndarray:
    cols = Columns(c.schema, X.shape[0], {f"f{j}": X[:, j] for j in range(N_FIELDS)})
    t, u = eval_predicate(p, cols)
    return np.where(u, SV_U, np.where(t, SV_T, SV_F))


def _check(c, p, X) -> bool:
    """True when the program was accepted (and then matched the oracle on every row)."""
    prog = compile_predicate(p, c)
    try:
        insns, pool, starts = predicate_programs([prog])
    except NotLowerable:
        assert postfix_depth(p) > SEG_STACK
        return False
    assert postfix_depth(p) <= SEG_STACK
    want = _oracle(c, p, X)
    got = np.array([kernel_model(insns, pool, int(starts[0]), X[r]) for r in range(X.shape[0])])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"row {bad[:5]}: kernel {got[bad[:5]]} vs oracle {want[bad[:5]]}"
    return True


def test_verdict_examples():
    """AND(20 x True, AND(20 x True)) needs 40 entries: refused (the kernel model shows the overflow
    would have read FALSE). OR(AND(20), AND(20)) peaks at 21: accepted and TRUE."""
    c = _doc()
    X = _inputs(8, 0)
    deep = ir.CompoundPredicate("and", [ir.TruePredicate()] * 20 +
                                [ir.CompoundPredicate("and", [ir.TruePredicate()] * 20)])
    assert postfix_depth(deep) == 40
    assert not _check(c, deep, X)
    # what the unguarded kernel would have done with it: the shift register lost the outer entries
    insns = [(1, 0, 0, 0)] * 20 + [(1, 0, 0, 0)] * 20 + [(7, 20, 0, 0), (7, 21, 0, 0), (0, 0, 0, 0)]
    assert kernel_model(insns, [0.0], 0, X[0]) == SV_F
    wide = ir.CompoundPredicate("or", [ir.CompoundPredicate("and", [ir.TruePredicate()] * 20)] * 2)
    assert postfix_depth(wide) == 21 and _check(c, wide, X)
    two32 = ir.CompoundPredicate("and", [ir.CompoundPredicate("or", [ir.TruePredicate()] * 32)] * 2)
    assert postfix_depth(two32) == 33 and not _check(c, two32, X)


def test_exact_limit_accepted():
    """A program that needs exactly SEG_STACK entries is the deepest the kernel takes."""
    c = _doc()
    p = ir.CompoundPredicate("xor", [ir.SimplePredicate(f"f{i % N_FIELDS}", "greaterThan", "0.1")
                                     for i in range(SEG_STACK)])
    assert _check(c, p, _inputs(64, 1))


@pytest.mark.parametrize("seed", range(8))
def test_random_nested_predicates_match_oracle(seed):
    rng = random.Random(seed)
    c = _doc()
    X = _inputs(32, seed)
    accepted = refused = 0
    for _ in range(200):
        p = random_predicate(rng, rng.randrange(1, 9))
        if _check(c, p, X):
            accepted += 1
        else:
            refused += 1
    assert accepted > 60 and refused > 0


@pytest.mark.parametrize("seed", range(4))
def test_wide_deep_predicates(seed):
    """Biased to overflow: wide compounds nested 2-4 deep, half refused, the rest exact."""
    rng = random.Random(100 + seed)
    c = _doc()
    X = _inputs(24, seed)
    seen = set()
    for _ in range(30):
        p = ir.CompoundPredicate(rng.choice(["and", "or", "xor", "surrogate"]),
                                 [random_predicate(rng, rng.randrange(1, 4), max_width=32)
                                  for _ in range(rng.randrange(8, 33))])
        seen.add(_check(c, p, X))
    assert False in seen  # the overflow side is exercised (accepted ones matched the oracle)


def to_xml(p: ir.Predicate) -> str:
    if isinstance(p, ir.TruePredicate):
        return "<True/>"
    if isinstance(p, ir.FalsePredicate):
        return "<False/>"
    if isinstance(p, ir.SimplePredicate):
        v = "" if p.value is None else f' value="{p.value}"'
        return f'<SimplePredicate field="{p.field}" operator="{p.operator}"{v}/>'
    if isinstance(p, ir.SimpleSetPredicate):
        return (f'<SimpleSetPredicate field="{p.field}" booleanOperator="{p.boolean_operator}">'
                f'<Array type="real" n="{len(p.values)}">{" ".join(p.values)}</Array></SimpleSetPredicate>')
    return (f'<CompoundPredicate booleanOperator="{p.boolean_operator}">'
            + "".join(to_xml(q) for q in p.predicates) + "</CompoundPredicate>")


def segmented_with_predicates(preds, method: str = "selectFirst", seed: int = 3) -> str:
    """``synth.segmented_pmml`` (fields f0..f5) with the first segments' predicates replaced."""
    from flink_jpmml_amd.bench.synth import segmented_pmml

    txt = segmented_pmml(method, False, n_segments=max(4, len(preds) + 1), seed=seed)
    for i, p in enumerate(preds):
        a = txt.index(f'<Segment id="{i + 1}"')
        j = txt.index(">", a) + 1
        k = txt.index("\n", j)
        txt = txt[:j] + to_xml(p) + txt[k:]
    return txt


def test_segmented_documents_with_deep_predicates_lower_or_refuse():
    """Whole documents: a 40-deep segment predicate keeps the tensor-op predicates (no fused
    reduction), a 32-deep one takes the fused kernel; both score like the oracle in the dry run."""
    import torch

    from flink_jpmml_amd.runtime.plans import compile_plan, lowering_dry_run

    deep = ir.CompoundPredicate("and", [ir.SimplePredicate("f0", "greaterThan", "-3")] * 20 +
                                [ir.CompoundPredicate("and", [ir.SimplePredicate("f1", "lessThan", "3")] * 20)])
    ok = ir.CompoundPredicate("or", [ir.SimplePredicate(f"f{i % 6}", "greaterThan", "0.3") for i in range(32)])
    for p, fused in ((deep, False), (ok, True)):
        c = CompiledPmml.from_string(segmented_with_predicates([p]))
        with lowering_dry_run():
            plan = compile_plan(c, torch.device("cpu"))
        plan = getattr(plan, "inner", plan)
        assert (plan._red is not None) == fused
