"""Randomized derived-field expressions through the derive program: random Apply trees (arithmetic,
n-ary aggregates, unary math incl. the PMML 4.4 functions, comparisons, if / isMissing, modulo,
hypot / atan2), NormContinuous, NormDiscrete, Discretize and MapValues over two continuous fields and
one categorical field, with random mapMissingTo / defaultValue attributes. CPU: the program's numpy
twin (`runtime/derive.py::emulate`) vs the float64 oracle's columns; GPU: the derive kernel vs the
twin, column for column (so a kernel bug cannot hide behind a model's aggregation)."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.runtime.compiled import CompiledPmml

NS = "http://www.dmg.org/PMML-4_4"
UNARY = ["abs", "floor", "ceil", "round", "sin", "cos", "tanh", "atan", "erf", "stdNormalCDF", "stdNormalPDF",
         "expm1", "rint"]
SAFE_UNARY = {"ln": "abs1", "sqrt": "abs", "ln1p": "abs", "log10": "abs1", "exp": "tanh"}  # guarded domains
BINARY = ["+", "-", "*", "/", "modulo", "hypot", "atan2", "min", "max"]
NARY = ["min", "max", "sum", "avg", "median", "product"]
COMPARE = ["equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual"]


def _const(rng) -> str:
    return f"<Constant>{rng.choice([0.0, 0.5, -1.25, 2.0, 3.0]) if rng.random() < 0.5 else round(rng.normal(), 3)}</Constant>"


def _attrs(rng) -> str:
    a = ""
    if rng.random() < 0.25:
        a += f' mapMissingTo="{round(rng.normal(), 2)}"'
    if rng.random() < 0.15:
        a += f' defaultValue="{round(rng.normal(), 2)}"'
    return a


def _expr(rng, depth: int, top: bool = False) -> str:
    r = rng.random()
    if depth == 0 or (r < 0.2 and not top):
        if rng.random() < 0.8:
            f = rng.choice(["a", "b"])
            mm = f' mapMissingTo="{round(rng.normal(), 2)}"' if rng.random() < 0.2 else ""
            return f'<FieldRef field="{f}"{mm}/>'
        return _const(rng)
    k = rng.integers(8)
    sub = lambda: _expr(rng, depth - 1)  # noqa: E731
    if k == 0:
        return f'<Apply function="{rng.choice(UNARY)}"{_attrs(rng)}>{sub()}</Apply>'
    if k == 1:
        fn, guard = list(SAFE_UNARY.items())[rng.integers(len(SAFE_UNARY))]
        inner = sub()
        if guard == "abs":
            inner = f'<Apply function="abs">{inner}</Apply>'
        elif guard == "abs1":
            inner = f'<Apply function="+"><Apply function="abs">{inner}</Apply><Constant>1</Constant></Apply>'
        else:
            inner = f'<Apply function="tanh">{inner}</Apply>'
        return f'<Apply function="{fn}"{_attrs(rng)}>{inner}</Apply>'
    if k == 2:
        return f'<Apply function="{rng.choice(BINARY)}"{_attrs(rng)}>{sub()}{sub()}</Apply>'
    if k == 3:
        n = int(rng.integers(2, 4))
        return f'<Apply function="{rng.choice(NARY)}"{_attrs(rng)}>{"".join(sub() for _ in range(n))}</Apply>'
    if k == 4:
        cond = f'<Apply function="{rng.choice(COMPARE)}">{sub()}{sub()}</Apply>'
        return f'<Apply function="if"{_attrs(rng)}>{cond}{sub()}{sub()}</Apply>'
    if k == 5:
        fn = rng.choice(["isMissing", "isNotMissing"])
        return f'<Apply function="{fn}"><FieldRef field="{rng.choice(["a", "b"])}"/></Apply>'
    if k == 6:
        return f'<Apply function="pow"{_attrs(rng)}>{sub()}<Constant>2</Constant></Apply>'
    return f'<Apply function="threshold">{sub()}{_const(rng)}</Apply>'


def _leaf_field(rng, i: int) -> str:
    """A derived field: a random Apply tree, or one of the other expression kinds."""
    k = rng.integers(10)
    name = f"d{i}"
    if k < 6:
        body = _expr(rng, int(rng.integers(2, 5)), top=True)
    elif k == 6:
        o = sorted(np.round(rng.normal(size=3), 2))
        if len(set(o)) < 3:
            o = [-1.0, 0.0, 1.0]
        outl = rng.choice(["asIs", "asMissingValues", "asExtremeValues"])
        body = (f'<NormContinuous field="{rng.choice(["a", "b"])}" outliers="{outl}"'
                f'{" mapMissingTo=" + chr(34) + "0.5" + chr(34) if rng.random() < 0.5 else ""}>'
                + "".join(f'<LinearNorm orig="{x}" norm="{j * 0.5}"/>' for j, x in enumerate(o)) + "</NormContinuous>")
    elif k == 7:
        body = f'<NormDiscrete field="c" value="{rng.choice(["red", "green", "blue"])}" mapMissingTo="-1"/>'
    elif k == 8:
        e = sorted(np.round(rng.normal(size=2), 2))
        body = (f'<Discretize field="a" mapMissingTo="9" defaultValue="7"><DiscretizeBin binValue="1"><Interval '
                f'closure="openClosed" rightMargin="{e[0]}"/></DiscretizeBin><DiscretizeBin binValue="2"><Interval '
                f'closure="openOpen" leftMargin="{e[0]}" rightMargin="{e[1] + 0.01}"/></DiscretizeBin></Discretize>')
    else:
        body = ('<MapValues outputColumn="out" defaultValue="0" mapMissingTo="-5"><FieldColumnPair field="c" '
                'column="col"/><InlineTable>'
                + "".join(f'<row><col>{v}</col><out>{round(rng.normal(), 2)}</out></row>'
                          for v in rng.permutation(["red", "green", "blue"])[:2]) + '</InlineTable></MapValues>')
    return f'  <DerivedField name="{name}" optype="continuous" dataType="double">{body}</DerivedField>\n'


N_FIELDS = 8


def _doc(seed: int) -> str:
    rng = np.random.default_rng(7000 + seed)
    fields = "".join(_leaf_field(rng, i) for i in range(N_FIELDS))
    preds = "".join(f'<NumericPredictor name="d{i}" coefficient="1"/>' for i in range(N_FIELDS))
    return (f'<PMML version="4.4" xmlns="{NS}"><DataDictionary>'
            '<DataField name="a" optype="continuous" dataType="double"/>'
            '<DataField name="b" optype="continuous" dataType="double"/>'
            '<DataField name="c" optype="categorical" dataType="string"><Value value="red"/><Value value="green"/>'
            '<Value value="blue"/></DataField><DataField name="y" optype="continuous" dataType="double"/>'
            f'</DataDictionary><TransformationDictionary>\n{fields}</TransformationDictionary>'
            '<RegressionModel functionName="regression"><MiningSchema><MiningField name="y" usageType="target"/>'
            '<MiningField name="a"/><MiningField name="b"/><MiningField name="c"/></MiningSchema>'
            f'<RegressionTable intercept="0">{preds}</RegressionTable></RegressionModel></PMML>')


def _inputs(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    X = np.empty((n, 3))
    X[:, 0] = rng.normal(0, 1.5, n)
    X[:, 1] = rng.normal(0.3, 1.0, n)
    X[:, 2] = rng.integers(0, 3, n)
    X[rng.random((n, 3)) < 0.08] = np.nan
    X[: n // 10, 1] = np.round(X[: n // 10, 1])  # ties for comparisons / modulo / rounding
    return X.astype(np.float32).astype(np.float64)


def _program(c):
    from flink_jpmml_amd.runtime.derive import plan_field_layout

    layout = plan_field_layout(c)
    assert layout.program is not None
    return layout.program


def _close_frac(got: np.ndarray, ref: np.ndarray) -> float:
    """Fraction of rows whose values differ beyond fp32 (NaN must match NaN)."""
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    both = ~nan_g & ~nan_r
    tol = 2e-6 * np.maximum(1.0, np.abs(ref))
    bad = (nan_g != nan_r) | (both & (np.abs(np.where(both, got - ref, 0.0)) > tol))
    return float(bad.mean())


@pytest.mark.parametrize("seed", range(60))
def test_program_twin_matches_oracle(seed):
    from flink_jpmml_amd.runtime.derive import emulate

    c = CompiledPmml.from_string(_doc(seed))
    prog = _program(c)
    X = _inputs(3000, seed)
    P, ok = c.prepare(X)
    got = emulate(prog, P).astype(np.float64)
    cols = c.columns(P)
    for j, name in enumerate(prog.selected):
        ref = cols.get(name).astype(np.float32).astype(np.float64)
        # discontinuous functions (floor, comparisons, bins) may flip on the rare fp32-rounded tie
        assert _close_frac(got[:, j], ref) <= 0.002, (seed, name)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(60, 16))
def test_derive_kernel_matches_twin(gpu, seed):
    import torch

    from flink_jpmml_amd.runtime.derive import DerivedPlan, emulate

    c = CompiledPmml.from_string(_doc(seed))
    plan = c.plan(gpu)
    assert isinstance(plan, DerivedPlan)
    X = _inputs(20_000, seed)
    P, _ = c.prepare(X)
    Xt = torch.from_numpy(X.astype(np.float32)).to(gpu)
    Xa, _ = plan._buffers(None, len(X))
    sc, va = plan.alloc_outputs(len(X))
    plan.launch(Xt, sc, va)
    torch.cuda.synchronize()
    dev = Xa.cpu().numpy().astype(np.float64)
    twin = emulate(plan.program, P).astype(np.float64)
    for j in range(dev.shape[1]):
        assert _close_frac(dev[:, j], twin[:, j]) <= 0.001, (seed, j)
