"""Derived fields on the device.

PMML documents usually compute the model's inputs from the raw record through
``TransformationDictionary`` / ``LocalTransformations`` ``DerivedField`` expressions (casts,
normalisations, discretisation, lookup tables, arithmetic). The reference hands the whole record
to JPMML, which evaluates them per record inside ``ModelEvaluator.evaluate``
(`S/api/PmmlModel.scala:143-160`). Here they are lowered once, at plan time, into one of two
forms (:func:`plan_field_layout`):

* **aliases** — a derived field that is a pure numeric cast of an input (``float(x)`` /
  ``double(x)`` ``FieldRef``, the XGBoost / LightGBM / sklearn2pmml idiom) is resolved to the
  input's column: the tree kernel reads the raw matrix, no extra pass;
* **folds** (tree ensembles) — a derived field that is a *monotone* function of one input
  (``(x - mu) / sd``, ``(c - x) * k``, ``NormContinuous`` with ``asIs`` / ``asExtremeValues``
  outliers, and chains of these) and that the model reads only as a tree split field: every
  split ``f(x) OP t`` is rewritten at lowering time into ``x < C`` or ``x >= C`` on the raw
  input, with ``C`` the fp32 cut found by bisecting the fp32 line against the float64 oracle's
  own evaluation of ``f`` (:func:`fold_splits`) — exact for every fp32 input, and the derive pass
  disappears (the transform is fused into the thresholds, zero device work);
* **program** — anything else becomes a postfix program over a per-row fp64 stack, run by
  ``ops/csrc/derive.hip`` in one memory-bound pass that also applies the MiningField
  preparation; it writes the ``[rows, columns the model reads]`` matrix that the model kernel
  consumes (:class:`DerivedPlan`).

The program mirrors :func:`flink_jpmml_amd.pmml.fields.eval_expression` (the float64 oracle)
instruction for instruction; :func:`emulate` is its numpy twin, used by the CPU tests to pin the
lowering against the oracle without a GPU. Stored columns are fp32 (as every model kernel
consumes); a ``double`` derived field that feeds *another* derived field is therefore rounded to
fp32 in between (the oracle keeps fp64) — the only numeric difference, documented in the tests.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..pmml import ir
from .plans import DevicePlan, NotLowerable, TreePlan, _addr

NAN = float("nan")
STACK_DEPTH = 16  # mirrors csrc/derive.hip::DSTACK
MAX_TILE_COLUMNS = 256  # LDS: 16 KiB stack + 128 rows x columns x 4 B <= 160 KiB

OP_LOAD, OP_CONST, OP_MAPMISS, OP_REMAP, OP_NORMCONT, OP_NORMDISC, OP_DISCRETIZE, OP_MAPVALUES, OP_APPLY, \
    OP_STORE = range(10)

APPLY_FN: Dict[str, int] = {
    "+": 0, "-": 1, "*": 2, "/": 3, "pow": 4, "modulo": 5, "hypot": 6, "atan2": 7,
    "equal": 10, "notEqual": 11, "lessThan": 12, "lessOrEqual": 13, "greaterThan": 14, "greaterOrEqual": 15,
    "threshold": 16,
    "log10": 20, "ln": 21, "sqrt": 22, "abs": 23, "exp": 24, "floor": 25, "ceil": 26, "round": 27, "rint": 28,
    "sin": 29, "cos": 30, "tan": 31, "asin": 32, "acos": 33, "atan": 34, "sinh": 35, "cosh": 36, "tanh": 37,
    "expm1": 38, "ln1p": 39, "not": 40, "x-exp": 24,
    "erf": 41, "stdNormalCDF": 42, "stdNormalPDF": 43, "stdNormalIDF": 44,
    "min": 50, "max": 51, "sum": 52, "avg": 53, "product": 54, "median": 55, "and": 56, "or": 57,
    "isMissing": 60, "isNotMissing": 61, "if": 62,
}
_BINARY_ARITH = range(0, 8)
_COMPARE = range(10, 17)
_UNARY = range(20, 45)
_OUTLIERS = {"asIs": 0, "asMissingValues": 1, "asExtremeValues": 2}

INSN_DTYPE = np.dtype([("op", "<i4"), ("a", "<i4"), ("b", "<i4"), ("c", "<i4"), ("x", "<f8"), ("y", "<f8")])


def _opt(v) -> float:
    return NAN if v is None else float(v)


# --------------------------------------------------------------------------- analysis


def _model_of(compiled) -> ir.Model:
    """The model IR the evaluator runs (Scorecard / RuleSet evaluate a rewritten tree IR)."""
    return getattr(compiled.evaluator, "model", None) or compiled.model


def collect_derived(compiled) -> Dict[str, ir.DerivedField]:
    """Every DerivedField visible to the model: TransformationDictionary + the LocalTransformations
    of the model and of all nested segment models (names must be unambiguous)."""
    out: Dict[str, ir.DerivedField] = {}

    def add(d: ir.DerivedField) -> None:
        prev = out.get(d.name)
        if prev is not None and prev != d:
            raise NotLowerable(f"derived field {d.name!r} is defined twice with different expressions")
        out[d.name] = d

    for d in compiled.doc.transformations:
        add(d)

    def walk(m: ir.Model) -> None:
        for d in m.local_transformations:
            add(d)
        if isinstance(m, ir.MiningModel):
            for s in m.segments:
                walk(s.model)

    walk(_model_of(compiled))
    return out


def _expr_fields(ex: ir.Expression, add) -> None:
    if isinstance(ex, (ir.FieldRef, ir.NormContinuous, ir.NormDiscrete, ir.Discretize)):
        add(ex.field)
    elif isinstance(ex, ir.MapValues):
        for f, _ in ex.field_columns:
            add(f)
    elif isinstance(ex, ir.Apply):
        for a in ex.args:
            _expr_fields(a, add)


def _pred_fields(p: ir.Predicate, add) -> None:
    if isinstance(p, (ir.SimplePredicate, ir.SimpleSetPredicate)):
        add(p.field)
    elif isinstance(p, ir.CompoundPredicate):
        for q in p.predicates:
            _pred_fields(q, add)


def referenced_fields(model: ir.Model) -> List[str]:
    """Field names the model element reads (document order, unique)."""
    seen: Dict[str, None] = {}

    def add(name: Optional[str]) -> None:
        if name is not None and name not in seen:
            seen[name] = None

    def walk(m: ir.Model) -> None:
        active = [f.name for f in m.mining_schema.active]
        if isinstance(m, ir.TreeModel) and m.flat is not None:
            for f in m.flat.field_names():
                add(f)
        elif isinstance(m, ir.TreeModel):
            stack = [m.root]
            while stack:
                nd = stack.pop()
                _pred_fields(nd.predicate, add)
                add(nd.value_field)
                stack.extend(reversed(nd.children))
        elif isinstance(m, ir.MiningModel):
            for s in m.segments:
                _pred_fields(s.predicate, add)
                walk(s.model)
        elif isinstance(m, ir.RegressionModel):
            for t in m.tables:
                for p in t.numeric:
                    add(p.name)
                for p in t.categorical:
                    add(p.name)
                for term in t.terms:
                    for f in term.fields:
                        add(f)
        elif isinstance(m, ir.ClusteringModel):
            fields = [f.field for f in m.fields if f.is_center_field] or active
            for f in fields:
                add(f)
        elif isinstance(m, ir.NeuralNetwork):
            for inp in m.inputs:
                _expr_fields(inp.derived.expression, add)
        elif isinstance(m, ir.SupportVectorMachineModel):
            for f in (m.vector_fields or active):
                add(f)
        else:  # GeneralRegression and anything else: its mining schema
            for f in active:
                add(f)

    walk(model)
    return list(seen)


def _deps(ex: ir.Expression) -> List[str]:
    out: List[str] = []
    _expr_fields(ex, out.append)
    return out


# --------------------------------------------------------------------------- lowering


@dataclass
class DerivedProgram:
    inputs: List[str]      # tile columns 0..F-1: the raw (prepared) active fields
    derived: List[str]     # tile columns F..: derived fields in evaluation order
    selected: List[str]    # columns handed to the model kernel, in order
    insns: np.ndarray      # INSN_DTYPE
    pool: np.ndarray       # float64 constant tables
    max_stack: int

    @property
    def n_tile(self) -> int:
        return len(self.inputs) + len(self.derived)

    @property
    def out_cols(self) -> np.ndarray:
        col = {n: i for i, n in enumerate(self.inputs + self.derived)}
        return np.array([col[n] for n in self.selected], dtype=np.int32)


class _Emitter:
    def __init__(self, schema, col_of: Dict[str, int]):
        self.schema = schema
        self.col_of = col_of
        self.insns: List[tuple] = []
        self.pool: List[float] = []
        self.sp = 0
        self.max_sp = 0

    def emit(self, op: int, a: int = 0, b: int = 0, c: int = 0, x: float = 0.0, y: float = 0.0,
             pops: int = 0, pushes: int = 0) -> None:
        self.insns.append((op, a, b, c, x, y))
        self.sp += pushes - pops
        self.max_sp = max(self.max_sp, self.sp)

    def table(self, values) -> int:
        off = len(self.pool)
        self.pool.extend(float(v) for v in values)
        return off

    def load(self, name: str) -> None:
        if name not in self.col_of:
            raise NotLowerable(f"field {name!r} is neither an input nor a lowered derived field")
        self.emit(OP_LOAD, a=self.col_of[name], pushes=1)

    # mirrors pmml/fields.py::eval_expression
    def expr(self, ex: ir.Expression, out_field: Optional[str]) -> None:
        s = self.schema
        if isinstance(ex, ir.Constant):
            if ex.missing or ex.value is None:
                v = NAN
            elif out_field is not None and s.is_string(out_field):
                v = float(s.code(out_field, ex.value))
            else:
                try:
                    v = float(ex.value)
                except ValueError:
                    v = float(s.code(out_field or "__const__", ex.value))
            self.emit(OP_CONST, x=v, pushes=1)
        elif isinstance(ex, ir.FieldRef):
            self.load(ex.field)
            if ex.map_missing_to is not None:
                self.emit(OP_MAPMISS, x=s.lookup(out_field or ex.field, ex.map_missing_to))
            if out_field is not None and s.is_string(out_field) and s.is_string(ex.field) and out_field != ex.field:
                remap = [s.code(out_field, v) for v in s.values.get(ex.field, [])]
                self.emit(OP_REMAP, a=self.table(remap), b=len(remap))
        elif isinstance(ex, ir.NormContinuous):
            orig = [ln.orig for ln in ex.norms]
            norm = [ln.norm for ln in ex.norms]
            if len(orig) < 2 or any(b <= a for a, b in zip(orig, orig[1:])):
                raise NotLowerable("NormContinuous needs >= 2 LinearNorms with increasing orig")
            self.load(ex.field)
            self.emit(OP_NORMCONT, a=self.table(orig + norm), b=len(orig), c=_OUTLIERS.get(ex.outliers, 0),
                      x=_opt(ex.map_missing_to))
        elif isinstance(ex, ir.NormDiscrete):
            self.load(ex.field)
            self.emit(OP_NORMDISC, x=s.lookup(ex.field, ex.value), y=_opt(ex.map_missing_to))
        elif isinstance(ex, ir.Discretize):
            self.load(ex.field)
            rows: List[float] = []
            tgt = out_field or "__bin__"
            for b in ex.bins:
                iv = b.interval
                clo = 0
                if iv.left is not None and not iv.closure.startswith("closed"):
                    clo |= 1
                if iv.right is not None and not iv.closure.endswith("Closed"):
                    clo |= 2
                if out_field:
                    val = s.lookup(tgt, b.bin_value)
                else:
                    try:
                        val = float(b.bin_value)
                    except ValueError as e:
                        raise NotLowerable("non-numeric Discretize bin in an anonymous expression") from e
                rows += [-math.inf if iv.left is None else iv.left, math.inf if iv.right is None else iv.right,
                         float(clo), val]
            mm = s.lookup(tgt, ex.map_missing_to) if ex.map_missing_to is not None else NAN
            dv = s.lookup(tgt, ex.default_value) if ex.default_value is not None else NAN
            self.emit(OP_DISCRETIZE, a=self.table(rows), b=len(ex.bins), x=mm, y=dv)
        elif isinstance(ex, ir.MapValues):
            tgt = out_field or "__map__"
            for fname, _ in ex.field_columns:
                self.load(fname)
            k = len(ex.field_columns)
            rows = []
            for row in ex.rows:
                for fname, colname in ex.field_columns:
                    rows.append(s.lookup(fname, row.get(colname)))
                rows.append(s.lookup(tgt, row.get(ex.output_column)))
            mm = s.lookup(tgt, ex.map_missing_to) if ex.map_missing_to is not None else NAN
            dv = s.lookup(tgt, ex.default_value) if ex.default_value is not None else NAN
            self.emit(OP_MAPVALUES, a=self.table(rows), b=len(ex.rows), c=k, x=mm, y=dv, pops=k, pushes=1)
        elif isinstance(ex, ir.Apply) and ex.function in ("isIn", "isNotIn") and ex.args \
                and isinstance(ex.args[0], ir.FieldRef) and ex.args[0].map_missing_to is None \
                and len(ex.args) > 1 and all(isinstance(a, ir.Constant) and not a.missing and a.value is not None
                                             for a in ex.args[1:]):
            # membership in a constant list = a one-column MapValues table (member -> 1 / 0, anything
            # else -> the default 0 / 1, a missing input -> mapMissingTo or missing)
            fname = ex.args[0].field
            self.load(fname)
            hit, other = (1.0, 0.0) if ex.function == "isIn" else (0.0, 1.0)
            rows = []
            for a in ex.args[1:]:
                rows += [s.lookup(fname, a.value), hit]
            try:
                mm = _opt(ex.map_missing_to)
            except ValueError as e:
                raise NotLowerable("non-numeric isIn mapMissingTo") from e
            self.emit(OP_MAPVALUES, a=self.table(rows), b=len(ex.args) - 1, c=1, x=mm, y=other, pops=1, pushes=1)
        elif isinstance(ex, ir.Apply):
            fn = ex.function
            fid = APPLY_FN.get(fn)
            n = len(ex.args)
            if fid is None:
                raise NotLowerable(f"Apply function {fn!r} is host-only")
            if (fid in _BINARY_ARITH and n != 2) or (fid in _COMPARE and n < 2) or n < 1 \
                    or (fid in _UNARY and fn not in ("not", "x-exp") and n != 1):
                raise NotLowerable(f"Apply {fn!r} with {n} arguments")
            for arg in ex.args:
                self.expr(arg, None)
            try:
                mm, dv = _opt(ex.map_missing_to), _opt(ex.default_value)
            except ValueError as e:
                raise NotLowerable("non-numeric Apply mapMissingTo/defaultValue") from e
            self.emit(OP_APPLY, a=fid, b=n, x=mm, y=dv, pops=n, pushes=1)
        else:
            raise NotLowerable(f"expression {type(ex).__name__} is host-only")


def _alias_source(name: str, defs: Dict[str, ir.DerivedField], inputs: Dict[str, int], schema) -> Optional[str]:
    """Input field a derived field is a lossless (on fp32 device inputs) numeric cast of, or None."""
    seen = set()
    while name in defs and name not in inputs:
        if name in seen:
            return None
        seen.add(name)
        d = defs[name]
        ex = d.expression
        if not isinstance(ex, ir.FieldRef) or ex.map_missing_to is not None:
            return None
        if d.data_type not in (None, "float", "double") or schema.is_string(ex.field):
            return None
        name = ex.field
    return name if name in inputs else None


def _monotone_expr(ex: ir.Expression, defs: Dict[str, ir.DerivedField], inputs: Dict[str, int], schema,
                   seen: set) -> Optional[str]:
    """Input field ``ex`` is a monotone (either direction), missing-preserving function of, or
    None. Accepted: casts, ``+`` / ``-`` / ``*`` with a constant, ``/`` by a non-zero constant,
    NormContinuous with strictly monotone norms and asIs / asExtremeValues outliers."""
    if isinstance(ex, ir.FieldRef):
        if ex.map_missing_to is not None or schema.is_string(ex.field):
            return None
        return _monotone_source(ex.field, defs, inputs, schema, seen)
    if isinstance(ex, ir.NormContinuous):
        norm = np.array([ln.norm for ln in ex.norms], dtype=np.float64)
        orig = np.array([ln.orig for ln in ex.norms], dtype=np.float64)
        if (ex.map_missing_to is not None or ex.outliers == "asMissingValues" or len(norm) < 2
                or not (np.diff(orig) > 0).all() or not ((np.diff(norm) > 0).all() or (np.diff(norm) < 0).all())
                or schema.is_string(ex.field)):
            return None
        return _monotone_source(ex.field, defs, inputs, schema, seen)
    if isinstance(ex, ir.Apply):
        if ex.map_missing_to is not None or ex.default_value is not None or len(ex.args) != 2 \
                or ex.function not in ("+", "-", "*", "/"):
            return None
        consts = [isinstance(a, ir.Constant) for a in ex.args]
        if consts.count(True) != 1:
            return None
        c = ex.args[consts.index(True)]
        try:
            cv = float(c.value)
        except (TypeError, ValueError):
            return None
        if c.missing or not math.isfinite(cv):
            return None
        if ex.function == "*" and cv == 0.0:
            return None
        if ex.function == "/" and (consts[0] or cv == 0.0):  # c / x is not monotone over the line
            return None
        return _monotone_expr(ex.args[consts.index(False)], defs, inputs, schema, seen)
    return None


def _monotone_source(name: str, defs: Dict[str, ir.DerivedField], inputs: Dict[str, int], schema,
                     seen: Optional[set] = None) -> Optional[str]:
    if name in inputs:
        return name
    seen = set() if seen is None else seen
    if name not in defs or name in seen:
        return None
    seen.add(name)
    d = defs[name]
    if d.data_type not in (None, "float", "double", "integer"):
        return None
    return _monotone_expr(d.expression, defs, inputs, schema, seen)


def _treated_fields(model: ir.Model) -> set:
    """Fields a (nested) MiningField prepares — missing / outlier / invalid treatment applied to
    the field's value itself: a derived field treated so can be neither aliased nor folded."""
    out: set = set()

    def walk(m: ir.Model) -> None:
        for mf in m.mining_schema.fields:
            if (mf.missing_value_replacement is not None or mf.outliers not in (None, "asIs")
                    or mf.invalid_value_treatment not in (None, "returnInvalid")):
                out.add(mf.name)
        if isinstance(m, ir.MiningModel):
            for sg in m.segments:
                walk(sg.model)

    walk(model)
    return out


def _non_split_refs(model: ir.Model) -> set:
    """Fields read anywhere but in a TreeModel node predicate (segment predicates, non-tree
    models), or treated by a MiningField: such a derived field cannot be folded into split
    thresholds."""
    out: set = _treated_fields(model)

    def walk(m: ir.Model) -> None:
        if isinstance(m, ir.TreeModel):
            return
        if isinstance(m, ir.MiningModel):
            for sg in m.segments:
                _pred_fields(sg.predicate, out.add)
                walk(sg.model)
            return
        out.update(referenced_fields(m))

    walk(model)
    return out


class FoldIndex(dict):
    """``field_index`` whose folded derived names map to their source input's column; ``folds``
    holds, per folded name, ``(source, f)`` with ``f`` the float64 oracle evaluation of the
    derived value from source values (:func:`fold_splits` rewrites the thresholds)."""

    def __init__(self, base: Dict[str, int], folds: Dict[str, tuple]):
        super().__init__(base)
        self.folds = folds


def _fold_fn(compiled, name: str, source: str, defs: Dict[str, ir.DerivedField]):
    from ..pmml.fields import Columns

    def f(xs: np.ndarray) -> np.ndarray:
        cols = Columns(compiled.schema, len(xs), {source: np.asarray(xs, dtype=np.float64)}, defs)
        return cols.get(name)

    return f


_F32_MAX_KEY = int(np.array(np.finfo(np.float32).max, np.float32).view(np.int32))


def _f32_from_key(k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, dtype=np.int64)
    bits = np.where(k < 0, (-k) | 0x80000000, k).astype(np.uint32)
    return bits.view(np.float32).astype(np.float64)


def fold_splits(f, ops: np.ndarray, ts: np.ndarray) -> tuple:
    """Rewrite splits ``f(x) OP t`` (OP codes of models/tree.py) on a monotone ``f`` into
    ``x < C`` (OP_LT) or ``x >= C`` (OP_GE) with fp32 ``C``, exact for every finite fp32 x: ``P(x)
    = f(x) OP t`` is monotone in x, so the cut is found by bisecting the ordered fp32 keys (33
    steps) with the oracle's ``f`` — vectorised over all splits of one field."""
    from ..models.tree import OP_GE, OP_GT, OP_LE, OP_LT

    ops = np.asarray(ops)
    ts = np.asarray(ts, dtype=np.float64)

    def P(x: np.ndarray) -> np.ndarray:
        y = f(x)
        return np.select([ops == OP_LT, ops == OP_LE, ops == OP_GT, ops == OP_GE],
                         [y < ts, y <= ts, y > ts, y >= ts], False)

    n = len(ts)
    lo = np.full(n, -_F32_MAX_KEY, np.int64)
    hi = np.full(n, _F32_MAX_KEY, np.int64)
    p_lo, p_hi = P(_f32_from_key(lo)), P(_f32_from_key(hi))
    rising = ~p_lo & p_hi   # P(x) <=> x >= C
    falling = p_lo & ~p_hi  # P(x) <=> x < C
    active = rising | falling
    for _ in range(34):
        if not active.any() or not (hi - lo > 1)[active].any():
            break
        mid = lo + (hi - lo) // 2
        pm = P(_f32_from_key(mid))
        below = np.where(rising, ~pm, pm)  # mid is still on lo's side of the cut
        lo = np.where(active & below & (hi - lo > 1), mid, lo)
        hi = np.where(active & ~below & (hi - lo > 1), mid, hi)
    cut = _f32_from_key(hi)
    new_ops = np.where(rising, OP_GE, OP_LT).astype(ops.dtype)
    # constant predicates: always true -> x < +inf, always false -> x < -inf
    new_t = np.where(active, cut, np.where(p_lo, np.inf, -np.inf))
    return new_ops, new_t


def _resolve_folds(model: ir.Model, folds: Dict[str, tuple]) -> None:
    """Fold every distinct ``(operator, value)`` split the model's trees make on each folded field
    in one vectorised bisection per field; ``folds[name]`` becomes ``(source, f, memo)`` with
    ``memo[(op, t)] = (op', t')`` for the tree lowering (exporters reuse split values heavily)."""
    from ..models.tree import _OPS

    want: Dict[str, Dict[tuple, None]] = {n: {} for n in folds}

    def walk(m: ir.Model) -> None:
        if isinstance(m, ir.TreeModel) and m.flat is not None and not m.flat.raw:
            from ..pmml.flat import OP_NAMES, P_SIMPLE

            a = m.flat.a
            simple = np.nonzero(a["pred_kind"] == P_SIMPLE)[0]
            for k in simple.tolist():
                name = m.flat.strings[int(a["pred_field"][k])]
                opn = OP_NAMES[int(a["pred_op"][k])]
                if name in want and opn in _OPS and not np.isnan(a["pred_value_d"][k]):
                    want[name][(_OPS[opn], float(a["pred_value_d"][k]))] = None
        elif isinstance(m, ir.TreeModel):
            stack = [m.root]
            while stack:
                nd = stack.pop()
                stack.extend(nd.children)
                p = nd.predicate
                if isinstance(p, ir.SimplePredicate) and p.field in want and p.operator in _OPS:
                    try:
                        want[p.field][(_OPS[p.operator], float(p.value))] = None
                    except (TypeError, ValueError):
                        pass
        elif isinstance(m, ir.MiningModel):
            for sg in m.segments:
                walk(sg.model)

    walk(model)
    for name, (src, f) in list(folds.items()):
        keys = list(want[name])
        memo = {}
        if keys:
            ops = np.array([k[0] for k in keys], np.int8)
            ts = np.array([k[1] for k in keys], np.float64)
            new_ops, new_ts = fold_splits(f, ops, ts)
            memo = {k: (int(o), float(t)) for k, o, t in zip(keys, new_ops, new_ts)}
        folds[name] = (src, f, memo)


@dataclass
class FieldLayout:
    columns: List[str]                 # the model kernel's input columns, in order
    field_index: Dict[str, int]        # every name the model may reference -> kernel column
    program: Optional[DerivedProgram]  # None: the kernel reads the raw input matrix
    evaluator: Optional[object] = None  # replaces the model's evaluator behind the view (design.py)
    folds: Optional[Dict[str, tuple]] = None  # folded derived names (tree split thresholds)


def plan_field_layout(compiled, allow_alias: bool = True, allow_fold: bool = False) -> FieldLayout:
    from ..models.tree import membership_fields

    active = list(compiled.active_fields)
    index = {f: i for i, f in enumerate(active)}
    defs = collect_derived(compiled)
    members = membership_fields(_model_of(compiled))  # 0/1 columns of categorical tree splits
    defs.update(members)
    if not defs:
        return FieldLayout(active, index, None)
    refs = referenced_fields(_model_of(compiled)) + list(members)
    shadow = [r for r in refs if r in defs and r in index]
    if shadow:  # a (local) derived field named like an input: the oracle's scope rules, not ours
        raise NotLowerable(f"derived field(s) {shadow} shadow input fields")
    needed = [r for r in refs if r in defs and r not in index]
    if not needed:
        return FieldLayout(active, index, None)
    schema = compiled.schema
    if allow_alias:
        treated = _treated_fields(_model_of(compiled))
        alias = {n: None if n in treated else _alias_source(n, defs, index, schema) for n in needed}
        folds: Dict[str, tuple] = {}
        if allow_fold and not all(v is not None for v in alias.values()):
            model = _model_of(compiled)
            blocked = _non_split_refs(model)
            for m in members.values():  # membership columns are computed from their field
                _expr_fields(m.expression, blocked.add)
            for n in needed:
                if alias[n] is None and n not in blocked and n not in members:
                    src = _monotone_source(n, defs, index, schema)
                    if src is not None:
                        folds[n] = (src, _fold_fn(compiled, n, src, defs))
        if folds:
            _resolve_folds(_model_of(compiled), folds)
        if all(v is not None or n in folds for n, v in alias.items()):
            fi = dict(index)
            fi.update({n: index[src] for n, src in alias.items() if src is not None})
            fi.update({n: index[fd[0]] for n, fd in folds.items()})
            return FieldLayout(active, fi, None, folds=folds or None)
    return build_program_layout(compiled, defs, refs)


def build_program_layout(compiled, defs: Dict[str, ir.DerivedField], refs: List[str]) -> FieldLayout:
    """Derive program computing every name of ``refs`` that is a derived field (inputs pass
    through); the kernel's columns are ``refs`` that resolve, in order."""
    active = list(compiled.active_fields)
    index = {f: i for i, f in enumerate(active)}
    schema = compiled.schema
    refs = list(dict.fromkeys(refs))
    needed = [r for r in refs if r in defs and r not in index]
    # evaluation order: depth-first post-order over the derived dependencies
    order: List[str] = []
    state: Dict[str, int] = {}

    def visit(name: str) -> None:
        if name in index or name not in defs:
            return
        st = state.get(name)
        if st == 2:
            return
        if st == 1:
            raise NotLowerable(f"cyclic derived field {name!r}")
        state[name] = 1
        for dep in _deps(defs[name].expression):
            visit(dep)
        state[name] = 2
        order.append(name)

    for n in needed:
        visit(n)
    if len(active) + len(order) > MAX_TILE_COLUMNS:
        raise NotLowerable(f"{len(active) + len(order)} input + derived columns > {MAX_TILE_COLUMNS}")
    col_of = dict(index)
    em = _Emitter(schema, col_of)
    for j, name in enumerate(order):
        d = defs[name]
        em.expr(d.expression, name)
        em.emit(OP_STORE, a=len(active) + j, c=2 if d.data_type == "integer" else 0, pops=1)
        col_of[name] = len(active) + j
    if em.max_sp > STACK_DEPTH:
        raise NotLowerable(f"derived expression needs a stack of {em.max_sp} > {STACK_DEPTH}")
    selected = [r for r in refs if r in col_of]
    insns = np.array(em.insns, dtype=INSN_DTYPE) if em.insns else np.zeros(0, INSN_DTYPE)
    prog = DerivedProgram(active, order, selected, insns, np.array(em.pool, dtype=np.float64), em.max_sp)
    return FieldLayout(selected, {n: i for i, n in enumerate(selected)}, prog)


# --------------------------------------------------------------------------- numpy twin (tests)


def emulate(prog: DerivedProgram, X: np.ndarray) -> np.ndarray:
    """numpy execution of the derive kernel on a *prepared* ``[rows, inputs]`` matrix; returns the
    ``[rows, selected]`` fp32 matrix the model kernel would read."""
    n = X.shape[0]
    tile = np.full((n, prog.n_tile), np.nan, dtype=np.float32)
    tile[:, : len(prog.inputs)] = np.asarray(X, dtype=np.float32)
    pool = prog.pool
    stack: List[np.ndarray] = []
    with np.errstate(all="ignore"):
        for op, a, b, c, x, y in prog.insns.tolist():
            if op == OP_LOAD:
                stack.append(tile[:, a].astype(np.float64))
            elif op == OP_CONST:
                stack.append(np.full(n, x))
            elif op == OP_MAPMISS:
                stack[-1] = np.where(np.isnan(stack[-1]), x, stack[-1])
            elif op == OP_REMAP:
                v = stack[-1]
                ok = ~np.isnan(v) & (v >= 0) & (v < b)
                tab = np.append(pool[a: a + b], NAN)
                stack[-1] = np.where(ok, tab[np.where(ok, v, b).astype(np.int64)], NAN)
            elif op == OP_NORMCONT:
                v = stack[-1]
                orig, nrm = pool[a: a + b], pool[a + b: a + 2 * b]
                seg = np.zeros(n, dtype=np.int64)
                for k in range(1, b - 1):
                    seg += v >= orig[k]
                r = nrm[seg] + (v - orig[seg]) * (nrm[seg + 1] - nrm[seg]) / (orig[seg + 1] - orig[seg])
                lo, hi = v < orig[0], v > orig[-1]
                if c == 1:
                    r = np.where(lo | hi, NAN, r)
                elif c == 2:
                    r = np.where(lo, nrm[0], np.where(hi, nrm[-1], r))
                stack[-1] = np.where(np.isnan(v), x, r)
            elif op == OP_NORMDISC:
                v = stack[-1]
                stack[-1] = np.where(np.isnan(v), y, (v == x).astype(np.float64))
            elif op == OP_DISCRETIZE:
                v = stack[-1]
                r = np.full(n, y)
                done = np.isnan(v)
                for k in range(b):
                    lo_, hi_, clo, val = pool[a + 4 * k: a + 4 * k + 4]
                    clo = int(clo)
                    m = ((v > lo_) if clo & 1 else (v >= lo_)) & ((v < hi_) if clo & 2 else (v <= hi_)) & ~done
                    r = np.where(m, val, r)
                    done |= m
                stack[-1] = np.where(np.isnan(v), x, r)
            elif op == OP_MAPVALUES:
                keys = stack[len(stack) - c:] if c else []
                del stack[len(stack) - c:]
                anymiss = np.zeros(n, dtype=bool)
                for kv in keys:
                    anymiss |= np.isnan(kv)
                r = np.full(n, y)
                matched = np.zeros(n, dtype=bool)
                for i in range(b):
                    row = pool[a + i * (c + 1): a + (i + 1) * (c + 1)]
                    m = ~matched & ~anymiss
                    for j, kv in enumerate(keys):
                        m &= kv == row[j]
                    r = np.where(m, row[c], r)
                    matched |= m
                stack.append(np.where(anymiss, x, r))
            elif op == OP_APPLY:
                args = stack[len(stack) - b:]
                del stack[len(stack) - b:]
                stack.append(_apply_np(a, args, x, y, n))
            elif op == OP_STORE:
                v = stack.pop()
                if c == 2:
                    v = np.where(np.isnan(v), v, np.trunc(v))
                tile[:, a] = v.astype(np.float32)
    return tile[:, prog.out_cols]


def _scipy(name: str):
    import scipy.special

    return getattr(scipy.special, name)


_NP_UNARY = {20: np.log10, 21: np.log, 22: np.sqrt, 23: np.abs, 24: np.exp, 25: np.floor, 26: np.ceil,
             27: lambda v: np.floor(v + 0.5), 28: np.rint, 29: np.sin, 30: np.cos, 31: np.tan, 32: np.arcsin,
             33: np.arccos, 34: np.arctan, 35: np.sinh, 36: np.cosh, 37: np.tanh, 38: np.expm1, 39: np.log1p,
             40: lambda v: (v == 0).astype(np.float64), 41: _scipy("erf"),
             42: lambda v: _scipy("ndtr")(v), 43: lambda v: np.exp(-0.5 * v * v) / np.sqrt(2.0 * np.pi),
             44: lambda v: _scipy("ndtri")(v)}
_NP_BINARY = {0: np.add, 1: np.subtract, 2: np.multiply, 3: np.divide, 4: np.power, 5: np.mod, 6: np.hypot,
              7: np.arctan2,
              10: np.equal, 11: np.not_equal, 12: np.less, 13: np.less_equal, 14: np.greater,
              15: np.greater_equal, 16: np.greater}
_NP_NARY = {50: np.nanmin, 51: np.nanmax, 52: np.nansum, 53: np.nanmean, 54: np.nanprod, 55: np.nanmedian}


def _apply_np(fn: int, args: List[np.ndarray], x: float, y: float, n: int) -> np.ndarray:
    if fn in (60, 61):
        m = np.isnan(args[0])
        return (m if fn == 60 else ~m).astype(np.float64)
    if fn == 62:
        cond = args[0]
        r = np.full(n, NAN)
        if len(args) > 1:
            r = np.where(cond == 1.0, args[1], r)
        if len(args) > 2:
            r = np.where(cond == 0.0, args[2], r)
        return r
    st = np.vstack(args)
    if fn in _NP_NARY:
        miss = np.all(np.isnan(st), axis=0)
        r = _NP_NARY[fn](np.where(miss[None, :], 0.0, st), axis=0)
    else:
        miss = np.any(np.isnan(st), axis=0)
        if fn in (56, 57):
            t = st != 0
            r = (np.all(t, axis=0) if fn == 56 else np.any(t, axis=0)).astype(np.float64)
        elif fn in _NP_UNARY:
            r = _NP_UNARY[fn](args[0])
        else:
            r = _NP_BINARY[fn](args[0], args[1]).astype(np.float64)
    r = np.asarray(r, dtype=np.float64)
    r = np.where(miss, x, r)
    return np.where(~miss & np.isnan(r) & ~np.isnan(y), y, r)


# --------------------------------------------------------------------------- views + plan


class FieldView:
    """A :class:`CompiledPmml` seen through a :class:`FieldLayout`: the model kernel's input columns
    (``active_fields``), the name → column map (``field_index``) and — when a derive pass ran
    first — inputs that are already prepared (no MiningField preparation in the model kernel)."""

    fields_resolved = True

    def __init__(self, compiled, layout: FieldLayout, prepared: bool):
        self._c = compiled
        self.active_fields = list(layout.columns)
        self.field_index = FoldIndex(layout.field_index, layout.folds) if layout.folds else dict(layout.field_index)
        self.folds = layout.folds
        self.prepared_inputs = prepared
        self.mining_fields = {} if prepared else dict(compiled.mining_fields)
        if layout.evaluator is not None:
            self.evaluator = layout.evaluator

    @property
    def n_features(self) -> int:
        return len(self.active_fields)

    def __getattr__(self, name):
        return getattr(self._c, name)


class DerivedPlan(DevicePlan):
    """derive kernel (prepare + derived fields) → model plan on the augmented matrix."""


    kind = "derived"
    _STATE = DevicePlan._STATE + ("insns", "pool", "out_cols", "n_tile", "n_sel", "n_insn", "supports_direct")

    def __init__(self, compiled, device, layout: FieldLayout, **opts):
        from .plans import compile_plan

        super().__init__(compiled, device)  # FieldPrep of the raw active fields
        prog = layout.program
        self.inner = compile_plan(FieldView(compiled, layout, prepared=True), device, **opts)
        self.insns = self._t(prog.insns.view(np.int32).reshape(-1))
        self.pool = self._t(prog.pool if prog.pool.size else np.zeros(1))
        self.out_cols = self._t(prog.out_cols)
        self.n_tile, self.n_sel, self.n_insn = prog.n_tile, len(prog.selected), len(prog.insns)
        self.supports_direct = bool(getattr(self.inner, "supports_direct", False))
        self.program = prog
        self._scratch = {}

    def _post_state(self) -> None:
        tensors = {k[6:]: v for k, v in self.__dict__.items() if k.startswith("inner/")}
        for k in list(self.__dict__):
            if k.startswith("inner/"):
                del self.__dict__[k]
        self.inner = DevicePlan.from_state(self.inner_meta, tensors, self.device)
        self._scratch = {}

    def export_state(self):
        meta, tensors = super().export_state()
        im, it = self.inner.export_state()
        meta["inner_meta"] = im
        for k, t in it.items():
            tensors["inner/" + k] = t
        meta["__tensors__"].update({"inner/" + k: v for k, v in im["__tensors__"].items()})
        return meta, tensors

    def _buffers(self, stream, n: int):
        """Per-stream scratch (allocated on that stream: reuse is stream-ordered)."""
        import torch

        from ..ops._lib import stream_handle

        key = stream_handle(stream)
        buf = self._scratch.get(key)
        if buf is None or buf[0].shape[0] < n:
            s = stream if stream is not None else torch.cuda.current_stream(self.device)
            with torch.cuda.stream(s):
                m = max(n, 1024)
                buf = (torch.empty((m, self.n_sel), dtype=torch.float32, device=self.device),
                       torch.empty(m, dtype=torch.uint8, device=self.device))
            self._scratch[key] = buf
        return buf[0][:n], buf[1][:n]

    def launch(self, X, score, valid, stream=None, probs=None, **kw) -> None:
        import ctypes

        from ..ops._lib import DeriveArgs, check, ptr, stream_handle

        n = X.shape[0]
        if n == 0:
            return
        Xa, ok = self._buffers(stream, n)
        a = DeriveArgs()
        a.X = X.data_ptr()
        a.n_rows, a.n_in, a.ldx, a.n_tile = n, X.shape[1], X.stride(0), self.n_tile
        a.prep, a.prog, a.pool, a.out_cols = ptr(self.prep), ptr(self.insns), ptr(self.pool), ptr(self.out_cols)
        a.n_insn, a.n_sel = self.n_insn, self.n_sel
        a.out, a.row_ok = ptr(Xa), ptr(ok)
        h = stream_handle(stream)
        check(self.lib.pmml_derive_launch(h, ctypes.byref(a)), "derive kernel")
        if isinstance(self.inner, TreePlan):
            self.inner.launch(Xa, score, valid, stream=stream, probs=probs, row_valid=ok, **kw)
            return
        self.inner.launch(Xa, score, valid, stream=stream, probs=probs, **kw)
        check(self.lib.pmml_mask_invalid(h, _addr(score), _addr(valid), ptr(ok), _addr(kw.get("score2")),
                                         _addr(kw.get("valid2")), n), "mask_invalid kernel")
