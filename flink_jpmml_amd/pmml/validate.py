"""Load-time checks of the literals a model compares its inputs against (fail closed).

JPMML parses a predicate's ``value`` into the field's data type when it evaluates it
(`S/api/PmmlModel.scala:159-160`); a literal that is not a number on a numeric field throws and
the reference turns the record into ``EmptyScore`` (`S/api/PmmlModel.scala:109-119`,
`S/models/prediction/Prediction.scala:47-62`). The engine encodes every value as a number before
any kernel runs, so such a literal cannot be carried to the rows that reach it: it would become a
vocabulary code (or NaN on the streaming-scanner path) and the model would score every row as a
valid ``Score``. A document with one is therefore rejected at load — :class:`PmmlParseError`, which
the operators turn into ``ModelLoadingException`` like any other malformed document.

Checked, on fields whose data type is numeric (``integer`` / ``float`` / ``double``) or
``boolean``:

* ``SimplePredicate`` comparison values (a missing ``value`` on a comparison operator is rejected
  for every data type), ``SimpleSetPredicate`` array members;
* ``NormDiscrete`` values and ``MapValues`` key cells;

over the whole document: transformation dictionary, every model's local transformations, tree
nodes (object trees and the scanner's flat arrays, ``pmml/flat.py``), segment, rule and scorecard
predicates. ``Array n=`` disagreeing with the number of entries is rejected by the parser
(``pmml/parser.py::_parse_array``). Numbers follow Java's ``Double.parseDouble`` grammar
(:func:`java_double_ok`): ``inf``, ``nan`` or ``1_000`` are not numbers to JPMML either.

Deviation (documented in ``docs/PARITY.md``): the reference fails only the records whose
evaluation reaches the bad literal (lazily, per record); here the whole document fails to load.
"""

from __future__ import annotations

import dataclasses
import re
from typing import Optional

import numpy as np

from ..api.exceptions import PmmlParseError
from . import ir

_NUMERIC = ("integer", "float", "double")
_COMPARE = ("equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual")


# java.lang.Double.parseDouble's decimal grammar (after its trim of characters <= U+0020):
# optional sign, then NaN / Infinity (exact case) or digits with an optional fraction and
# exponent. Python's float() also accepts "inf", "nan", "infinity" in any case and "1_000", which
# Java rejects; Java's type suffixes (1.5f, 2d) and hex floats (0x1p3) are not accepted here either
# (float() cannot read them, and no exporter writes them): such documents fail closed.
_JAVA_DOUBLE = re.compile(r"[+-]?(NaN|Infinity|(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)")


def java_double_ok(value: str) -> bool:
    """Whether ``value`` parses as a Java double (the JPMML number grammar) and as a Python float
    with the same value."""
    v = value.strip(" \t\n\r\x0b\x0c\x00")
    return bool(_JAVA_DOUBLE.fullmatch(v))


def literal_ok(data_type: Optional[str], value: Optional[str]) -> bool:
    """Whether ``value`` is a literal of a field typed ``data_type`` (untyped / string: any)."""
    if data_type not in _NUMERIC and data_type != "boolean":
        return True
    if value is None:
        return False
    if data_type == "boolean" and value.strip().lower() in ("true", "false"):
        return True
    if not java_double_ok(value):
        return False
    try:
        float(value)
    except ValueError:
        return False
    return True


class _Checker:
    def __init__(self, schema):
        self.schema = schema

    def dtype(self, name: str) -> Optional[str]:
        return self.schema.types.get(name)

    def literal(self, what: str, fld: str, value: Optional[str]) -> None:
        t = self.dtype(fld)
        if not literal_ok(t, value):
            raise PmmlParseError(f"{what} on {t} field {fld!r}: value {value!r} is not a {t}")

    def visit(self, obj) -> None:
        stack = [obj]
        while stack:
            o = stack.pop()
            if isinstance(o, (list, tuple)):
                stack.extend(o)
                continue
            if isinstance(o, dict) or not dataclasses.is_dataclass(o):
                continue
            if isinstance(o, ir.SimplePredicate):
                if o.operator in _COMPARE:
                    if o.value is None:
                        raise PmmlParseError(f"SimplePredicate {o.operator} on {o.field!r} has no value")
                    self.literal(f"SimplePredicate {o.operator}", o.field, o.value)
                continue
            if isinstance(o, ir.SimpleSetPredicate):
                for v in o.values:
                    self.literal(f"SimpleSetPredicate {o.boolean_operator}", o.field, v)
                continue
            if isinstance(o, ir.NormDiscrete):
                self.literal("NormDiscrete", o.field, o.value)
                continue
            if isinstance(o, ir.MapValues):
                for fld, col in o.field_columns:
                    for row in o.rows:
                        v = row.get(col)
                        if v is not None:
                            self.literal(f"MapValues column {col!r}", fld, v)
                continue
            if isinstance(o, ir.TreeModel):
                stack.extend((o.mining_schema, o.output, o.targets, o.local_transformations))
                if o.flat is not None:
                    self.flat(o.flat)
                elif o.root is not None:
                    stack.append(o.root)
                continue
            for f in dataclasses.fields(o):
                v = getattr(o, f.name, None)
                if isinstance(v, (list, tuple)) or dataclasses.is_dataclass(v):
                    stack.append(v)

    def flat(self, ft) -> None:
        """The scanner's node arrays: simple predicates are (field, operator, value string) columns;
        compound / set predicates were parsed into ``ft.raw_pred``."""
        a = ft.a
        if ft.n:
            cmp = (a["pred_kind"] == 2) & (a["pred_op"] < len(_COMPARE))  # flat.P_SIMPLE, OP_NAMES[:6]
            fld = a["pred_field"][cmp].astype(np.int64)
            val = a["pred_value_s"][cmp].astype(np.int64)
            if fld.size:
                pairs = np.unique(np.stack([fld, val], axis=1), axis=0)
                for f, v in pairs.tolist():
                    name = ft.strings[f]
                    if v < 0:
                        raise PmmlParseError(f"SimplePredicate on {name!r} has no value")
                    self.literal("SimplePredicate", name, ft.strings[v])
        self.visit(list(ft.raw_pred.values()))


def validate_literals(doc: ir.PMMLDocument, schema) -> None:
    """Raise :class:`PmmlParseError` for a literal its field's data type cannot hold (module doc).
    ``schema`` must have every model registered (``FieldSchema.register_model``), so local derived
    fields are typed."""
    c = _Checker(schema)
    c.visit(list(doc.transformations))
    c.visit(doc.model)


__all__ = ["literal_ok", "validate_literals"]
