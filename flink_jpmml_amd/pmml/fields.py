"""Field typing, value preparation and the columnar evaluation context.

Every value the engine touches is encoded as a ``float64`` (host oracle) / ``float32`` (device):

* continuous / numeric categorical / boolean fields: the number itself;
* string-typed fields: an integer *code* into a per-field vocabulary (``FieldSchema.vocab``),
  seeded from the ``DataDictionary`` valid values in document order (so ordinal comparisons on
  codes follow the declared order) and extended with every literal the model mentions;
* missing values: ``NaN``.

That uniform ``[rows, fields]`` float matrix is exactly what the HIP kernels consume, so the CPU
oracle and the GPU path share one data model.

Preparation follows the PMML/JPMML rules the reference relies on through
``EvaluatorUtil.prepare`` (`S/api/PmmlModel.scala:143-152`): missing-value detection and
replacement, type conversion, validity (intervals / valid values) with ``invalidValueTreatment``
and ``outliers`` handling from the ``MiningField``.
"""

from __future__ import annotations

import math
import re
from typing import Any, Callable, Dict, Iterable, List, Optional

import numpy as np

from ..api.exceptions import EvaluationException, InputPreparationException, UnsupportedFeatureException
from . import ir

NAN = float("nan")
_NUMERIC_TYPES = ("integer", "float", "double", "boolean")


class InvalidValue(Exception):
    """A value is invalid under ``invalidValueTreatment="returnInvalid"``."""


class FieldSchema:
    """Document-wide field typing + string vocabularies."""

    def __init__(self, doc: ir.PMMLDocument):
        self.doc = doc
        self.data_fields: Dict[str, ir.DataField] = dict(doc.data_fields)
        self.derived: Dict[str, ir.DerivedField] = {d.name: d for d in doc.transformations}
        self.types: Dict[str, str] = {}
        self.optypes: Dict[str, str] = {}
        self.vocab: Dict[str, Dict[str, int]] = {}
        self.values: Dict[str, List[str]] = {}
        for df in self.data_fields.values():
            self.types[df.name] = df.data_type
            self.optypes[df.name] = df.optype
            if df.is_string:
                for v in df.values:
                    self.code(df.name, v)
        for d in doc.transformations:
            self._register_derived(d)

    # ------------------------------------------------------------------ typing
    def _register_derived(self, d: ir.DerivedField) -> None:
        self.derived.setdefault(d.name, d)
        if d.data_type:
            self.types.setdefault(d.name, d.data_type)
        if d.optype:
            self.optypes.setdefault(d.name, d.optype)
        if self.is_string(d.name):
            for v in d.values:
                self.code(d.name, v)

    def register_model(self, model: ir.Model) -> None:
        for d in model.local_transformations:
            self._register_derived(d)
        for of in model.output:
            if of.data_type:
                self.types.setdefault(of.name, of.data_type)
            elif of.feature in ("predictedValue", "predictedDisplayValue") and of.target_field:
                self.types.setdefault(of.name, self.types.get(of.target_field, "double"))
            if of.feature in ("entityId", "clusterId", "predictedDisplayValue", "reasonCode", "warning"):
                self.types.setdefault(of.name, "string")

    def is_string(self, name: str) -> bool:
        return self.types.get(name) == "string"

    def code(self, name: str, value: str) -> int:
        voc = self.vocab.setdefault(name, {})
        c = voc.get(value)
        if c is None:
            c = len(voc)
            voc[value] = c
            self.values.setdefault(name, []).append(value)
        return c

    def lookup(self, name: str, value: str) -> float:
        """Literal ``value`` (as written in the PMML) converted into the field's encoding."""
        if self.is_string(name):
            return float(self.code(name, value))
        if value is None:
            return NAN
        if self.types.get(name) == "boolean":
            lv = value.strip().lower()
            if lv in ("true", "1"):
                return 1.0
            if lv in ("false", "0"):
                return 0.0
        try:
            return float(value)
        except ValueError:
            # a string literal compared against a numeric field: give the field a vocabulary
            return float(self.code(name, value))

    def decode(self, name: str, v: float) -> Any:
        if v is None or (isinstance(v, float) and math.isnan(v)):
            return None
        if self.is_string(name):
            vals = self.values.get(name, [])
            i = int(v)
            return vals[i] if 0 <= i < len(vals) else None
        t = self.types.get(name)
        if t == "integer":
            return int(v)
        if t == "boolean":
            return bool(v)
        return float(v)

    # ------------------------------------------------------------------ prepare
    def prepare_value(self, name: str, raw: Any, mf: Optional[ir.MiningField]) -> float:
        """Prepare one raw input value into the field's numeric encoding (NaN = missing).

        Raises :class:`InvalidValue` for an invalid value under ``returnInvalid`` and
        :class:`InputPreparationException` when the field definition itself cannot accept values.
        """
        df = self.data_fields.get(name)
        dtype = df.data_type if df is not None else self.types.get(name, "double")
        optype = (mf.optype if mf is not None and mf.optype else None) or (df.optype if df is not None else "continuous")
        if df is not None and optype != "continuous" and df.intervals:
            # An Interval only makes sense on a continuous field (JPMML rejects the field).
            raise InputPreparationException(f"field {name!r}: Interval is not allowed on a {optype} field")
        is_missing = raw is None or (isinstance(raw, float) and math.isnan(raw))
        if not is_missing and df is not None and df.missing_values and _in_value_list(df, raw, df.missing_values):
            is_missing = True
        value = NAN
        if not is_missing:
            try:
                value = self._convert(name, dtype, raw)
                valid = self._is_valid(df, optype, raw, value)
            except InvalidValue:
                valid = False
            if not valid:
                treatment = mf.invalid_value_treatment if mf is not None else "returnInvalid"
                if treatment in ("asIs",):
                    if math.isnan(value):
                        value = self._force_code(name, raw)
                elif treatment == "asMissing":
                    is_missing = True
                    value = NAN
                elif treatment == "asValue" and mf is not None and mf.invalid_value_replacement is not None:
                    value = self._convert(name, dtype, mf.invalid_value_replacement)
                else:
                    raise InvalidValue(f"field {name!r}: invalid value {raw!r}")
            elif mf is not None and optype == "continuous" and not math.isnan(value):
                value = _apply_outliers(value, mf)
                if math.isnan(value):
                    is_missing = True
        if is_missing or math.isnan(value):
            if mf is not None and mf.missing_value_replacement is not None:
                return self._convert(name, dtype, mf.missing_value_replacement)
            return NAN
        return value

    def _force_code(self, name: str, raw: Any) -> float:
        if self.is_string(name):
            return float(self.code(name, _as_text(raw)))
        try:
            return float(raw)
        except (TypeError, ValueError):
            return NAN

    def _convert(self, name: str, dtype: str, raw: Any) -> float:
        if dtype == "string":
            return float(self.code(name, _as_text(raw)))
        if dtype == "boolean":
            if isinstance(raw, str):
                s = raw.strip().lower()
                if s in ("true", "1", "1.0"):
                    return 1.0
                if s in ("false", "0", "0.0"):
                    return 0.0
                raise InvalidValue(f"not a boolean: {raw!r}")
            return 1.0 if float(raw) != 0 else 0.0
        try:
            v = float(raw)
        except (TypeError, ValueError) as e:
            raise InvalidValue(f"field {name!r}: {raw!r} is not a {dtype}") from e
        if dtype == "integer" and v != math.floor(v):
            raise InvalidValue(f"field {name!r}: {raw!r} is not an integer")
        if dtype == "float":
            v = float(np.float32(v))
        return v

    def _is_valid(self, df: Optional[ir.DataField], optype: str, raw: Any, value: float) -> bool:
        if df is None:
            return True
        if df.invalid_values and _in_value_list(df, raw, df.invalid_values):
            return False
        if optype == "continuous":
            if df.intervals and not any(iv.contains(value) for iv in df.intervals):
                return False
            if df.values and not df.is_string:
                return any(_num_eq(value, v) for v in df.values) or bool(df.intervals)
            return True
        if df.values:
            if df.is_string:
                return _as_text(raw) in df.values
            return any(_num_eq(value, v) for v in df.values)
        return True

    # ---------------------------------------------------------- batch prepare
    def prepare_matrix(self, names: List[str], X: np.ndarray, mfs: Dict[str, ir.MiningField]) -> tuple:
        """Vectorised prepare of a numeric ``[rows, len(names)]`` matrix (NaN = missing).

        Returns ``(prepared, row_valid)``. Only numeric encodings are handled here (string fields
        must already be coded); it implements missing replacement, intervals + invalid
        treatment and outliers — the same semantics as :meth:`prepare_value`.
        """
        X = np.array(X, dtype=np.float64, copy=True)
        valid = np.ones(X.shape[0], dtype=bool)
        float_cols, general = self._prep_plan(names, mfs)
        if len(float_cols):
            # fields with no preparation besides the float data type's rounding, in one op
            X[:, float_cols] = X[:, float_cols].astype(np.float32).astype(np.float64)
        for j, name in general:
            col = X[:, j]
            mf = mfs.get(name)
            df = self.data_fields.get(name)
            optype = (mf.optype if mf is not None and mf.optype else None) or (df.optype if df else "continuous")
            if df is not None and optype != "continuous" and df.intervals:
                valid[:] = False
                continue
            miss = np.isnan(col)
            present = ~miss
            if df is not None and df.missing_values and not df.is_string:
                for mv in df.missing_values:
                    try:
                        miss |= col == float(mv)
                    except ValueError:
                        pass
                present = ~miss
            bad = np.zeros_like(miss)
            if df is not None and df.invalid_values and not df.is_string:
                for iv in df.invalid_values:
                    try:
                        bad |= present & (col == float(iv))
                    except ValueError:
                        pass
            if df is not None and optype == "continuous" and df.intervals:
                inside = np.zeros_like(miss)
                for iv in df.intervals:
                    inside |= _interval_mask(iv, col)
                bad |= present & ~inside
            elif df is not None and df.values and optype != "continuous":
                if df.is_string:
                    allowed = np.arange(len(df.values), dtype=np.float64)
                else:
                    allowed = np.array([float(v) for v in df.values])
                bad |= present & ~np.isin(col, allowed)
            if df is not None and df.data_type == "integer":
                bad |= present & (np.floor(col) != col)
            if bad.any():
                treat = mf.invalid_value_treatment if mf is not None else "returnInvalid"
                if treat == "asMissing":
                    miss |= bad
                elif treat == "asValue" and mf is not None and mf.invalid_value_replacement is not None:
                    col[bad] = float(mf.invalid_value_replacement)
                elif treat != "asIs":
                    valid &= ~bad
            if mf is not None and optype == "continuous":
                # outlier treatment belongs to the VALID-value treatment (as in prepare_value and
                # JPMML): invalid values kept asIs or replaced asValue are not clamped / voided
                ok_vals = present & ~bad
                if mf.outliers == "asMissingValues":
                    if mf.low_value is not None:
                        miss |= ok_vals & (col < mf.low_value)
                    if mf.high_value is not None:
                        miss |= ok_vals & (col > mf.high_value)
                elif mf.outliers == "asExtremeValues":
                    if mf.low_value is not None:
                        col[ok_vals & (col < mf.low_value)] = mf.low_value
                    if mf.high_value is not None:
                        col[ok_vals & (col > mf.high_value)] = mf.high_value
            col[miss] = NAN
            if mf is not None and mf.missing_value_replacement is not None:
                col[miss] = self.lookup(name, mf.missing_value_replacement)
            if df is not None and df.data_type == "float":
                X[:, j] = col.astype(np.float32).astype(np.float64)
            else:
                X[:, j] = col
        return X, valid

    def _prep_plan(self, names: List[str], mfs: Dict[str, ir.MiningField]) -> tuple:
        """Split ``names`` into the columns :meth:`prepare_matrix` leaves as they are (at most a
        float32 rounding) and the ones that need the per-field treatment; cached per name list
        and MiningField map, so per-record calls skip the per-field checks."""
        cache = self.__dict__.setdefault("_prep_plans", {})
        key = tuple(names)
        hit = cache.get(key)
        if hit is not None and hit[0] is mfs:
            return hit[1], hit[2]
        float_cols, general = [], []
        for j, name in enumerate(names):
            mf = mfs.get(name)
            df = self.data_fields.get(name)
            optype = (mf.optype if mf is not None and mf.optype else None) or (df.optype if df else "continuous")
            trivial = (
                (mf is None or (mf.missing_value_replacement is None
                                and (optype != "continuous" or mf.outliers not in ("asMissingValues", "asExtremeValues"))))
                and (df is None or (not df.missing_values and not df.invalid_values and not df.intervals
                                    and not (df.values and optype != "continuous")
                                    and df.data_type != "integer")))
            if not trivial:
                general.append((j, name))
            elif df is not None and df.data_type == "float":
                float_cols.append(j)
        plan = (np.asarray(float_cols, dtype=np.intp), general)
        cache[key] = (mfs,) + plan
        return plan


def _in_value_list(df: ir.DataField, raw: Any, values: List[str]) -> bool:
    """Membership of a raw input in a DataField's missing / invalid Value list: by text, and for
    numeric fields by value too (-999.0 matches "-999", as the typed comparison of JPMML and the
    matrix path ``prepare_matrix`` do)."""
    if _as_text(raw) in values:
        return True
    if df.is_string:
        return False
    try:
        x = float(raw)
    except (TypeError, ValueError):
        return False
    for v in values:
        try:
            if float(v) == x:
                return True
        except ValueError:
            continue
    return False


def _as_text(raw: Any) -> str:
    if isinstance(raw, str):
        return raw
    if isinstance(raw, bool):
        return "true" if raw else "false"
    if isinstance(raw, float) and raw.is_integer():
        # Java's Double.toString(1.0) == "1.0"; keep that for categorical matching parity
        return repr(raw)
    return str(raw)


def _num_eq(v: float, lit: str) -> bool:
    try:
        return v == float(lit)
    except ValueError:
        return False


def _apply_outliers(v: float, mf: ir.MiningField) -> float:
    if mf.outliers == "asMissingValues":
        if (mf.low_value is not None and v < mf.low_value) or (mf.high_value is not None and v > mf.high_value):
            return NAN
    elif mf.outliers == "asExtremeValues":
        if mf.low_value is not None and v < mf.low_value:
            return mf.low_value
        if mf.high_value is not None and v > mf.high_value:
            return mf.high_value
    return v


def _interval_mask(iv: ir.Interval, col: np.ndarray) -> np.ndarray:
    m = np.ones(col.shape, dtype=bool)
    with np.errstate(invalid="ignore"):
        if iv.left is not None:
            m &= (col >= iv.left) if iv.closure.startswith("closed") else (col > iv.left)
        if iv.right is not None:
            m &= (col <= iv.right) if iv.closure.endswith("Closed") else (col < iv.right)
    return m


# --------------------------------------------------------------------------- columnar context


class Columns:
    """Lazy column store: ``name -> float64[n]`` with derived fields computed on first access."""

    def __init__(self, schema: FieldSchema, n: int, base: Optional[Dict[str, np.ndarray]] = None,
                 derived: Optional[Dict[str, ir.DerivedField]] = None):
        self.schema = schema
        self.n = n
        self.data: Dict[str, np.ndarray] = dict(base or {})
        self.derived: Dict[str, ir.DerivedField] = dict(schema.derived)
        if derived:
            self.derived.update(derived)
        self._busy: set = set()
        # the [n, k] matrix the base columns are views of, and name -> column (CompiledPmml.columns);
        # lets a consumer of many base columns take them in one gather (None once a base column is
        # replaced through set())
        self.matrix: Optional[np.ndarray] = None
        self.mindex: Optional[Dict[str, int]] = None

    def child(self, extra_derived: Iterable[ir.DerivedField], rows: Optional[np.ndarray] = None) -> "Columns":
        """A context for a nested model; shares computed columns (optionally row-subset)."""
        ders = {d.name: d for d in extra_derived}
        if rows is None:
            c = Columns(self.schema, self.n, self.data, {**self.derived, **ders})
        else:
            c = Columns(self.schema, int(len(rows)), {k: v[rows] for k, v in self.data.items()},
                        {**self.derived, **ders})
        return c

    def has(self, name: str) -> bool:
        return name in self.data or name in self.derived

    def get(self, name: str) -> np.ndarray:
        col = self.data.get(name)
        if col is not None:
            return col
        d = self.derived.get(name)
        if d is None:
            raise EvaluationException(f"field {name!r} is not defined")
        if name in self._busy:
            raise EvaluationException(f"cyclic derived field {name!r}")
        self._busy.add(name)
        try:
            col = eval_expression(d.expression, self, out_field=name)
            if d.data_type == "float":
                col = col.astype(np.float32).astype(np.float64)
            elif d.data_type == "integer":
                col = np.where(np.isnan(col), col, np.trunc(col))
        finally:
            self._busy.discard(name)
        self.data[name] = col
        return col

    def set(self, name: str, col: np.ndarray) -> None:
        if self.mindex is not None and name in self.mindex:
            self.matrix = None
        self.data[name] = col


# --------------------------------------------------------------------------- expressions


def _arr(n: int, v: float) -> np.ndarray:
    return np.full(n, v, dtype=np.float64)


def eval_expression(ex: ir.Expression, cols: Columns, out_field: Optional[str] = None) -> np.ndarray:
    n = cols.n
    schema = cols.schema
    if isinstance(ex, ir.Constant):
        if ex.missing or ex.value is None:
            return _arr(n, NAN)
        if out_field is not None and schema.is_string(out_field):
            return _arr(n, float(schema.code(out_field, ex.value)))
        try:
            return _arr(n, float(ex.value))
        except ValueError:
            return _arr(n, float(schema.code(out_field or "__const__", ex.value)))
    if isinstance(ex, ir.FieldRef):
        col = cols.get(ex.field)
        if ex.map_missing_to is not None:
            col = np.where(np.isnan(col), schema.lookup(out_field or ex.field, ex.map_missing_to), col)
        if out_field is not None and schema.is_string(out_field) and schema.is_string(ex.field) and out_field != ex.field:
            src_vals = schema.values.get(ex.field, [])
            remap = np.array([schema.code(out_field, v) for v in src_vals], dtype=np.float64)
            ok = ~np.isnan(col)
            res = _arr(n, NAN)
            if len(remap):
                res[ok] = remap[col[ok].astype(np.int64)]
            return res
        return col
    if isinstance(ex, ir.NormContinuous):
        x = cols.get(ex.field)
        return norm_continuous(ex, x)
    if isinstance(ex, ir.NormDiscrete):
        x = cols.get(ex.field)
        lit = schema.lookup(ex.field, ex.value)
        res = (x == lit).astype(np.float64)
        miss = np.isnan(x)
        res[miss] = NAN if ex.map_missing_to is None else ex.map_missing_to
        return res
    if isinstance(ex, ir.Discretize):
        x = cols.get(ex.field)
        res = _arr(n, NAN)
        done = np.isnan(x)
        for b in ex.bins:
            m = ~done & _interval_mask(b.interval, x)
            res[m] = schema.lookup(out_field or "__bin__", b.bin_value) if out_field else float(b.bin_value)
            done |= m
        miss = np.isnan(x)
        if ex.map_missing_to is not None:
            res[miss] = schema.lookup(out_field or "__bin__", ex.map_missing_to)
        rest = ~done
        if ex.default_value is not None:
            res[rest] = schema.lookup(out_field or "__bin__", ex.default_value)
        return res
    if isinstance(ex, ir.MapValues):
        keys = []
        for fname, colname in ex.field_columns:
            keys.append((cols.get(fname), fname, colname))
        res = _arr(n, NAN)
        matched = np.zeros(n, dtype=bool)
        anymiss = np.zeros(n, dtype=bool)
        for arr, _, _ in keys:
            anymiss |= np.isnan(arr)
        tgt = out_field or "__map__"
        for row in ex.rows:
            m = ~matched & ~anymiss
            for arr, fname, colname in keys:
                m &= arr == schema.lookup(fname, row.get(colname))
            if m.any():
                res[m] = schema.lookup(tgt, row.get(ex.output_column))
                matched |= m
        if ex.map_missing_to is not None:
            res[anymiss] = schema.lookup(tgt, ex.map_missing_to)
        if ex.default_value is not None:
            res[~matched & ~anymiss] = schema.lookup(tgt, ex.default_value)
        return res
    if isinstance(ex, ir.Apply):
        return _eval_apply(ex, cols, out_field)
    raise UnsupportedFeatureException(f"expression {type(ex).__name__} not supported")


def norm_continuous(ex: ir.NormContinuous, x: np.ndarray) -> np.ndarray:
    norms = ex.norms
    if len(norms) < 2:
        raise EvaluationException("NormContinuous needs at least two LinearNorm elements")
    orig = np.array([ln.orig for ln in norms])
    norm = np.array([ln.norm for ln in norms])
    res = np.empty_like(x)
    miss = np.isnan(x)
    xs = np.where(miss, orig[0], x)
    lo, hi = xs < orig[0], xs > orig[-1]
    # inner segments: piecewise-linear interpolation
    seg = np.clip(np.searchsorted(orig, xs, side="right") - 1, 0, len(orig) - 2)
    x0, x1 = orig[seg], orig[seg + 1]
    y0, y1 = norm[seg], norm[seg + 1]
    res = y0 + (xs - x0) * (y1 - y0) / (x1 - x0)
    if ex.outliers == "asMissingValues":
        res[lo | hi] = NAN
    elif ex.outliers == "asExtremeValues":
        res[lo] = norm[0]
        res[hi] = norm[-1]
    res[miss] = NAN if ex.map_missing_to is None else ex.map_missing_to
    return res


def denorm_continuous(ex: ir.NormContinuous, y: np.ndarray) -> np.ndarray:
    """Inverse of :func:`norm_continuous` (NeuralNetwork regression outputs)."""
    orig = np.array([ln.orig for ln in ex.norms])
    norm = np.array([ln.norm for ln in ex.norms])
    order = np.argsort(norm, kind="stable")
    norm_s, orig_s = norm[order], orig[order]
    seg = np.clip(np.searchsorted(norm_s, y, side="right") - 1, 0, len(norm_s) - 2)
    y0, y1 = norm_s[seg], norm_s[seg + 1]
    x0, x1 = orig_s[seg], orig_s[seg + 1]
    return x0 + (y - y0) * (x1 - x0) / (y1 - y0)


def _erf(a):
    from scipy.special import erf

    return erf(a)


def _ndtri(a):
    from scipy.special import ndtri

    return ndtri(a)


_SQRT2 = math.sqrt(2.0)
_SQRT2PI = math.sqrt(2.0 * math.pi)

_BINARY_NUM: Dict[str, Callable] = {
    "+": np.add, "-": np.subtract, "*": np.multiply, "/": np.divide, "pow": np.power,
    "min": np.fmin, "max": np.fmax, "modulo": np.mod, "hypot": np.hypot, "atan2": np.arctan2,
}
# PMML 4.4 distribution functions: f(x, mean, stdev)
_TERNARY_NUM: Dict[str, Callable] = {
    "normalCDF": lambda x, m, s: 0.5 * (1.0 + _erf((x - m) / (s * _SQRT2))),
    "normalPDF": lambda x, m, s: np.exp(-0.5 * ((x - m) / s) ** 2) / (s * _SQRT2PI),
    "normalIDF": lambda p, m, s: m + s * _ndtri(p),
}
_UNARY_NUM: Dict[str, Callable] = {
    "log10": np.log10, "ln": np.log, "sqrt": np.sqrt, "abs": np.abs, "exp": np.exp, "floor": np.floor,
    "ceil": np.ceil, "round": lambda a: np.floor(a + 0.5), "rint": np.rint, "sin": np.sin, "cos": np.cos,
    "tan": np.tan, "asin": np.arcsin, "acos": np.arccos, "atan": np.arctan, "sinh": np.sinh, "cosh": np.cosh,
    "tanh": np.tanh, "expm1": np.expm1, "ln1p": np.log1p, "erf": _erf,
    "stdNormalCDF": lambda a: 0.5 * (1.0 + _erf(a / _SQRT2)),
    "stdNormalPDF": lambda a: np.exp(-0.5 * a * a) / _SQRT2PI,
    "stdNormalIDF": _ndtri,
}


# String built-ins of the PMML function library (JPMML-Evaluator's FunctionRegistry): evaluated over
# decoded row strings, the result re-encoded into the output field's vocabulary.
_STRING_FUNCS = ("uppercase", "lowercase", "substring", "trimBlanks", "concat", "replace", "formatNumber")


def _text(v: Any) -> Optional[str]:
    if v is None or (isinstance(v, float) and math.isnan(v)):
        return None
    if isinstance(v, float):
        return str(int(v)) if v.is_integer() else repr(v)
    return str(v)


def _to_number(v: str) -> float:
    try:
        return float(v)
    except ValueError:
        return NAN


def eval_strings(ex: ir.Expression, cols: Columns) -> List[Optional[str]]:
    """Row-wise string values of ``ex`` (``None`` = missing): string fields decode their codes,
    numbers are written as in a document (3.0 -> ``3``), string built-ins apply row by row."""
    n = cols.n
    schema = cols.schema
    if isinstance(ex, ir.Constant):
        v = None if ex.missing else ex.value
        return [v] * n
    if isinstance(ex, ir.FieldRef):
        col = cols.get(ex.field)
        out = [_text(schema.decode(ex.field, float(c))) for c in col]
        if ex.map_missing_to is not None:
            out = [ex.map_missing_to if o is None else o for o in out]
        return out
    if isinstance(ex, ir.Apply) and ex.function in _STRING_FUNCS:
        return _apply_strings(ex, cols)
    col = eval_expression(ex, cols)
    return [_text(float(c)) for c in col]


def _apply_strings(ex: ir.Apply, cols: Columns) -> List[Optional[str]]:
    fn = ex.function
    n = cols.n
    if fn == "formatNumber":
        x = eval_expression(ex.args[0], cols)
        pat = eval_strings(ex.args[1], cols)
        out = []
        for v, p in zip(x, pat):
            if math.isnan(v) or p is None:
                out.append(None)
                continue
            try:
                out.append(p % (int(v) if re.search(r"%[-+ 0#]*\d*[dxXo]", p) else v))
            except (TypeError, ValueError):
                out.append(None)
        return out
    args = [eval_strings(a, cols) for a in ex.args]
    out: List[Optional[str]] = []
    for i in range(n):
        a = [arg[i] for arg in args]
        if fn == "concat":  # missing arguments are skipped (JPMML: null-safe concatenation)
            parts = [x for x in a if x is not None]
            out.append("".join(parts) if parts else None)
            continue
        if a[0] is None:
            out.append(None)
            continue
        if fn == "uppercase":
            out.append(a[0].upper())
        elif fn == "lowercase":
            out.append(a[0].lower())
        elif fn == "trimBlanks":
            out.append(a[0].strip())
        elif fn == "substring":  # substring(s, start (1-based), length)
            try:
                st, ln = int(float(a[1])), int(float(a[2]))
            except (TypeError, ValueError):
                out.append(None)
                continue
            out.append(a[0][max(st - 1, 0): max(st - 1, 0) + max(ln, 0)])
        elif fn == "replace":  # replace(s, regex, replacement)
            if a[1] is None or a[2] is None:
                out.append(None)
            else:
                out.append(re.sub(a[1], re.sub(r"\$(\d)", r"\\\1", a[2]), a[0]))
    return out


def _eval_apply(ex: ir.Apply, cols: Columns, out_field: Optional[str]) -> np.ndarray:
    n = cols.n
    fn = ex.function
    if fn in _STRING_FUNCS:
        vals = _apply_strings(ex, cols)
        if ex.map_missing_to is not None:
            vals = [ex.map_missing_to if v is None else v for v in vals]
        name = out_field or "__string__"
        if out_field is not None and not cols.schema.is_string(out_field):
            return np.array([NAN if v is None else _to_number(v) for v in vals], dtype=np.float64)
        return np.array([NAN if v is None else float(cols.schema.code(name, v)) for v in vals], dtype=np.float64)
    if fn == "matches":  # matches(s, regex): boolean
        s_, pat = eval_strings(ex.args[0], cols), eval_strings(ex.args[1], cols)
        return np.array([NAN if a is None or b is None else float(re.search(b, a) is not None)
                         for a, b in zip(s_, pat)], dtype=np.float64)
    if fn in ("isIn", "isNotIn"):  # isIn(field, value, value, ...): membership in the constant list
        x = eval_strings(ex.args[0], cols)
        members = set()
        for a in ex.args[1:]:
            if isinstance(a, ir.Constant) and not a.missing and a.value is not None:
                members.add(a.value)
                try:
                    members.add(_text(float(a.value)))
                except ValueError:
                    pass
            else:
                raise UnsupportedFeatureException(f"{fn}: only constant member lists are supported")
        hit = np.array([v is not None and v in members for v in x])
        res = hit if fn == "isIn" else ~hit
        res = res.astype(np.float64)
        res[np.array([v is None for v in x], dtype=bool)] = NAN
        if ex.map_missing_to is not None:
            res = np.where(np.isnan(res), float(ex.map_missing_to), res)
        return res
    args = [eval_expression(a, cols) for a in ex.args]
    with np.errstate(all="ignore"):
        if fn in ("isMissing", "isNotMissing"):
            m = np.isnan(args[0])
            res = (m if fn == "isMissing" else ~m).astype(np.float64)
            return res
        if fn == "if":
            cond = args[0]
            res = _arr(n, NAN)
            t = cond == 1.0
            res[t] = args[1][t] if len(args) > 1 else NAN
            if len(args) > 2:
                f = cond == 0.0
                res[f] = args[2][f]
            return res
        miss = np.zeros(n, dtype=bool)
        for a in args:
            miss |= np.isnan(a)
        if fn in _UNARY_NUM and len(args) == 1:
            res = _UNARY_NUM[fn](args[0])
        elif fn in ("+", "-", "*", "/", "pow", "modulo", "hypot", "atan2") and len(args) == 2:
            res = _BINARY_NUM[fn](args[0], args[1])
        elif fn in _TERNARY_NUM and len(args) == 3:
            res = _TERNARY_NUM[fn](args[0], args[1], args[2])
        elif fn == "stdev" and args:  # sample standard deviation of the present arguments
            stack = np.vstack(args)
            cnt = np.sum(~np.isnan(stack), axis=0)
            mean = np.nansum(stack, axis=0) / np.maximum(cnt, 1)
            ss = np.nansum((stack - mean) ** 2, axis=0)
            res = np.where(cnt >= 2, np.sqrt(ss / np.maximum(cnt - 1, 1)), NAN)
            miss = cnt == 0
        elif fn in ("min", "max", "sum", "avg", "product", "median") and args:
            stack = np.vstack(args)
            res = {"min": np.nanmin, "max": np.nanmax, "sum": np.nansum, "avg": np.nanmean, "product": np.nanprod,
                   "median": np.nanmedian}[fn](stack, axis=0)
            miss = np.all(np.isnan(stack), axis=0)
        elif fn in ("equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual"):
            op = {"equal": np.equal, "notEqual": np.not_equal, "lessThan": np.less, "lessOrEqual": np.less_equal,
                  "greaterThan": np.greater, "greaterOrEqual": np.greater_equal}[fn]
            res = op(args[0], args[1]).astype(np.float64)
        elif fn in ("and", "or"):
            stack = np.vstack(args) != 0
            res = (np.all(stack, axis=0) if fn == "and" else np.any(stack, axis=0)).astype(np.float64)
        elif fn == "not":
            res = (args[0] == 0).astype(np.float64)
        elif fn == "threshold":
            res = (args[0] > args[1]).astype(np.float64)
        elif fn == "x-exp":
            res = np.exp(args[0])
        else:
            raise UnsupportedFeatureException(f"Apply function {fn!r} not supported")
    res = np.asarray(res, dtype=np.float64)
    res = np.where(miss, NAN, res)
    if ex.map_missing_to is not None:
        res = np.where(miss, float(ex.map_missing_to), res)
    if ex.default_value is not None:
        res = np.where(np.isnan(res) & ~miss, float(ex.default_value), res)
    return res


# --------------------------------------------------------------------------- predicates
# Three-valued logic on numpy arrays: (true_mask, unknown_mask); false = ~true & ~unknown.


def eval_predicate(p: ir.Predicate, cols: Columns) -> tuple:
    n = cols.n
    if isinstance(p, ir.TruePredicate):
        return np.ones(n, dtype=bool), np.zeros(n, dtype=bool)
    if isinstance(p, ir.FalsePredicate):
        return np.zeros(n, dtype=bool), np.zeros(n, dtype=bool)
    if isinstance(p, ir.SimplePredicate):
        x = cols.get(p.field)
        miss = np.isnan(x)
        op = p.operator
        if op == "isMissing":
            return miss.copy(), np.zeros(n, dtype=bool)
        if op == "isNotMissing":
            return ~miss, np.zeros(n, dtype=bool)
        v = cols.schema.lookup(p.field, p.value)
        with np.errstate(invalid="ignore"):
            if op == "equal":
                t = x == v
            elif op == "notEqual":
                t = x != v
            elif op == "lessThan":
                t = x < v
            elif op == "lessOrEqual":
                t = x <= v
            elif op == "greaterThan":
                t = x > v
            elif op == "greaterOrEqual":
                t = x >= v
            else:
                raise UnsupportedFeatureException(f"SimplePredicate operator {op!r}")
        return t & ~miss, miss
    if isinstance(p, ir.SimpleSetPredicate):
        x = cols.get(p.field)
        miss = np.isnan(x)
        vals = np.array([cols.schema.lookup(p.field, v) for v in p.values], dtype=np.float64)
        inside = np.isin(x, vals)
        t = inside if p.boolean_operator == "isIn" else ~inside
        return t & ~miss, miss
    if isinstance(p, ir.CompoundPredicate):
        op = p.boolean_operator
        parts = [eval_predicate(q, cols) for q in p.predicates]
        if op == "surrogate":
            t = np.zeros(n, dtype=bool)
            u = np.ones(n, dtype=bool)
            for pt, pu in parts:
                take = u & ~pu
                t = np.where(take, pt, t)
                u = u & pu
            return t, u
        if op == "and":
            anyfalse = np.zeros(n, dtype=bool)
            anyunk = np.zeros(n, dtype=bool)
            for pt, pu in parts:
                anyfalse |= ~pt & ~pu
                anyunk |= pu
            t = ~anyfalse & ~anyunk
            return t, anyunk & ~anyfalse
        if op == "or":
            anytrue = np.zeros(n, dtype=bool)
            anyunk = np.zeros(n, dtype=bool)
            for pt, pu in parts:
                anytrue |= pt
                anyunk |= pu
            return anytrue, anyunk & ~anytrue
        if op == "xor":
            acc = np.zeros(n, dtype=bool)
            unk = np.zeros(n, dtype=bool)
            for pt, pu in parts:
                acc ^= pt
                unk |= pu
            return acc & ~unk, unk
        raise UnsupportedFeatureException(f"CompoundPredicate operator {op!r}")
    raise UnsupportedFeatureException(f"predicate {type(p).__name__}")
