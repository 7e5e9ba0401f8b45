"""Native (C++) execution of the float64 oracle's tree walk.

The oracle's :meth:`TreeEvaluator.leaf_index` walks a tree with numpy masks: exact, but one Python
iteration per node, so a 1000-tree GBDT scores ~1 k records/s on the host — the speed of every
``fallback="host"`` model, every direct CPU ``predict`` and the replay path. The reference runs
the same walk in compiled code (JPMML on the JVM, `S/api/PmmlModel.scala:159-160`).

:class:`ForestProgram` lowers one or many :class:`TreeEvaluator` s into flat int32 / float64
tables (``native/csrc/tree_walk.cpp`` documents the layout) that the ``_fastpath`` extension walks
row by row over the oracle's own prepared float64 columns. Every predicate is the oracle's
(three-valued logic, the same literal encoding through :meth:`FieldSchema.lookup`), every missing
value follows the same ``missingValueStrategy`` / ``noTrueChildStrategy`` rule, so the chosen
node is the numpy walk's by construction — ``tests/test_native_walk.py`` pins it on the reference
fixtures and on randomised trees (every predicate kind, every strategy, missing values).

A tree the builder cannot encode exactly (an unknown predicate type, a literal whose encoding
would grow a string vocabulary at evaluation time) returns ``None``: it keeps the numpy walk.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..pmml import ir

PK_TRUE, PK_FALSE, PK_SIMPLE, PK_IS_MISSING, PK_IS_NOT_MISSING = 0, 1, 2, 3, 4
PK_SET_IN, PK_SET_NOT_IN, PK_AND, PK_OR, PK_XOR, PK_SURROGATE = 5, 6, 7, 8, 9, 10
_SIMPLE_OPS = {"equal": 0, "notEqual": 1, "lessThan": 2, "lessOrEqual": 3, "greaterThan": 4, "greaterOrEqual": 5}
_FAST_OPS = {"lessThan": 0, "lessOrEqual": 1, "greaterThan": 2, "greaterOrEqual": 3}
_NEG = {"lessThan": "greaterOrEqual", "lessOrEqual": "greaterThan", "greaterThan": "lessOrEqual",
        "greaterOrEqual": "lessThan"}
_COMPOUND = {"and": PK_AND, "or": PK_OR, "xor": PK_XOR, "surrogate": PK_SURROGATE}
_STRATEGY = {"none": 0, "lastPrediction": 1, "defaultChild": 2, "nullPrediction": 3,
             "weightedConfidence": 3, "aggregateNodes": 3}
MAX_PRED_DEPTH = 48


class NotNative(Exception):
    """This tree keeps the numpy walk."""


def _pure_literal(schema, field: str, value) -> float:
    """:meth:`FieldSchema.lookup` without its side effect: a literal that is not yet in a string
    vocabulary would be appended to it when the numpy walk reaches the predicate — that tree stays
    on the numpy walk so vocabulary codes are assigned in the oracle's order."""
    if schema.is_string(field):
        voc = schema.vocab.get(field, {})
        if value in voc:
            return float(voc[value])
        raise NotNative(f"literal {value!r} not in the vocabulary of {field!r}")
    if value is None:
        return math.nan
    if schema.types.get(field) == "boolean":
        lv = value.strip().lower()
        if lv in ("true", "1"):
            return 1.0
        if lv in ("false", "0"):
            return 0.0
    try:
        return float(value)
    except ValueError:
        voc = schema.vocab.get(field, {})
        if value in voc:
            return float(voc[value])
        raise NotNative(f"non-numeric literal {value!r} for {field!r}") from None


class ForestProgram:
    """Flat tables of one or many trees (appended with :meth:`add`), plus the field list whose
    prepared columns form the walker's input matrix."""

    def __init__(self, schema):
        self.schema = schema
        self.fields: List[str] = []
        self._slot: Dict[str, int] = {}
        self.nodes_i: List[List[int]] = []
        self.nodes_d: List[float] = []
        self.kids: List[int] = []
        self.preds_i: List[List[int]] = []
        self.preds_d: List[float] = []
        self.aux_i: List[int] = []
        self.aux_d: List[float] = []
        self.roots: List[int] = []
        self.modes: List[int] = []
        self.n_nodes: List[int] = []
        self.leafval: List[np.ndarray] = []
        self._arrays = None

    # ------------------------------------------------------------------ building
    def field(self, name: str) -> int:
        s = self._slot.get(name)
        if s is None:
            s = self._slot[name] = len(self.fields)
            self.fields.append(name)
        return s

    def _pred(self, p: ir.Predicate, depth: int = 0) -> int:
        if depth > MAX_PRED_DEPTH:
            raise NotNative("predicate nesting too deep")
        pid = len(self.preds_i)
        if isinstance(p, ir.TruePredicate):
            self.preds_i.append([PK_TRUE, 0, 0, 0])
            self.preds_d.append(0.0)
        elif isinstance(p, ir.FalsePredicate):
            self.preds_i.append([PK_FALSE, 0, 0, 0])
            self.preds_d.append(0.0)
        elif isinstance(p, ir.SimplePredicate):
            op = p.operator
            if op in ("isMissing", "isNotMissing"):
                kind = PK_IS_MISSING if op == "isMissing" else PK_IS_NOT_MISSING
                self.preds_i.append([kind, 0, self.field(p.field), 0])
                self.preds_d.append(0.0)
            elif op in _SIMPLE_OPS:
                lit = _pure_literal(self.schema, p.field, p.value)
                self.preds_i.append([PK_SIMPLE, _SIMPLE_OPS[op], self.field(p.field), 0])
                self.preds_d.append(lit)
            else:
                raise NotNative(f"SimplePredicate operator {op!r}")
        elif isinstance(p, ir.SimpleSetPredicate):
            if p.boolean_operator not in ("isIn", "isNotIn"):
                raise NotNative(f"SimpleSetPredicate operator {p.boolean_operator!r}")
            vals = [_pure_literal(self.schema, p.field, v) for v in p.values]
            start = len(self.aux_i)
            self.aux_i.extend([len(vals), len(self.aux_d)])
            self.aux_d.extend(vals)
            kind = PK_SET_IN if p.boolean_operator == "isIn" else PK_SET_NOT_IN
            self.preds_i.append([kind, 0, self.field(p.field), start])
            self.preds_d.append(0.0)
        elif isinstance(p, ir.CompoundPredicate):
            kind = _COMPOUND.get(p.boolean_operator)
            if kind is None:
                raise NotNative(f"CompoundPredicate operator {p.boolean_operator!r}")
            self.preds_i.append([kind, 0, 0, 0])  # placeholder: children are encoded first
            self.preds_d.append(0.0)
            kids = [self._pred(q, depth + 1) for q in p.predicates]
            start = len(self.aux_i)
            self.aux_i.append(len(kids))
            self.aux_i.extend(kids)
            self.preds_i[pid][3] = start
        else:
            raise NotNative(f"predicate {type(p).__name__}")
        return pid

    def _fast(self, node: ir.Node):
        """``(field slot, op code, value, complement)`` for the exporters' binary split, else None."""
        if len(node.children) != 2:
            return None
        pa, pb = node.children[0].predicate, node.children[1].predicate
        if not isinstance(pa, ir.SimplePredicate) or pa.operator not in _FAST_OPS or \
                self.schema.is_string(pa.field):
            return None
        try:
            v = _pure_literal(self.schema, pa.field, pa.value)
        except NotNative:
            return None
        if math.isnan(v):
            return None
        if isinstance(pb, ir.TruePredicate):
            comp = False
        elif isinstance(pb, ir.SimplePredicate) and pb.field == pa.field and pb.operator == _NEG[pa.operator] \
                and pb.value == pa.value:
            comp = True
        else:
            return None
        return self.field(pa.field), _FAST_OPS[pa.operator], v, comp

    def add(self, ev, leafval: Optional[np.ndarray] = None) -> bool:
        """Append ``ev``'s tree (node order = ``ev.nodes``); False (nothing appended) if the tree
        cannot be encoded exactly."""
        mark = (len(self.nodes_i), len(self.kids), len(self.preds_i), len(self.aux_i), len(self.aux_d),
                len(self.fields))
        try:
            self._add(ev)
        except NotNative:
            n0, k0, p0, a0, d0, f0 = mark
            del self.nodes_i[n0:], self.nodes_d[n0:], self.kids[k0:], self.preds_i[p0:], self.preds_d[p0:]
            del self.aux_i[a0:], self.aux_d[d0:]
            for name in self.fields[f0:]:
                del self._slot[name]
            del self.fields[f0:]
            return False
        if leafval is not None:
            self.leafval.append(np.asarray(leafval, dtype=np.float64))
        self._arrays = None
        return True

    def _add(self, ev) -> None:
        tm = ev.tree
        strat = _STRATEGY.get(tm.missing_value_strategy)
        if strat is None:
            raise NotNative(f"missingValueStrategy {tm.missing_value_strategy!r}")
        nodes = ev.nodes
        index = ev._index
        base = len(self.nodes_i)
        for nd in nodes:
            self.nodes_i.append([0, 0, -1, 0, 0, 0, 0, -1])
            self.nodes_d.append(0.0)
        for i, nd in enumerate(nodes):
            rec = self.nodes_i[base + i]
            rec[7] = self._pred(nd.predicate)
            if not nd.children:
                continue
            ch = [base + index[id(c)] for c in nd.children]
            rec[0], rec[1] = len(ch), len(self.kids)
            self.kids.extend(ch)
            if nd.default_child is not None:
                for c in nd.children:
                    if c.id == nd.default_child:
                        rec[2] = base + index[id(c)]
                        break
            fast = self._fast(nd)
            if fast is not None:
                slot, op, v, comp = fast
                rec[3] = 1 | (op << 1) | (8 if comp else 0)
                rec[4], rec[5], rec[6] = slot, ch[0], ch[1]
                self.nodes_d[base + i] = v
        self.roots.append(base)
        self.modes.append(strat | ((1 if tm.no_true_child_strategy == "returnLastPrediction" else 0) << 4))
        self.n_nodes.append(len(nodes))

    # ------------------------------------------------------------------ running
    def arrays(self):
        if self._arrays is None:
            def i32(x, w=None):
                a = np.asarray(x, dtype=np.int32)
                return a.reshape(-1, w) if w and a.size else a.reshape(-1)

            lv = np.concatenate(self.leafval) if self.leafval else np.zeros(0)
            self._arrays = (i32(self.nodes_i).reshape(-1), np.asarray(self.nodes_d, dtype=np.float64),
                            i32(self.kids), i32(self.preds_i).reshape(-1), np.asarray(self.preds_d, dtype=np.float64),
                            i32(self.aux_i if self.aux_i else [0]), np.asarray(self.aux_d or [0.0], dtype=np.float64),
                            i32(self.roots), i32(self.modes), lv)
        return self._arrays

    def compiled(self):
        """The walker's fixed-depth / perfect tables of this program, built once (a capsule tied
        to the :meth:`arrays` buffers) so per-record calls do not rebuild them."""
        cap = getattr(self, "_capsule", None)
        if cap is None or cap[0] is not self._arrays:
            from ..native import fastpath

            arrs = self.arrays()
            ni, nd, kids, pi, pd, ai, ad, roots, modes, _ = arrs
            cap = (arrs, fastpath().forest_compile(ni, nd, kids, pi, pd, ai, ad, roots, modes,
                                                   max(1, len(self.fields))))
            self._capsule = cap
        return cap[1]

    @property
    def n_trees(self) -> int:
        return len(self.roots)

    def matrix(self, cols) -> np.ndarray:
        """The walker's input: the prepared float64 column of every referenced field, row-major.
        Raises whatever ``cols.get`` raises (the caller then keeps the numpy walk)."""
        n, k = cols.n, max(1, len(self.fields))
        M, mindex = getattr(cols, "matrix", None), getattr(cols, "mindex", None)
        if M is not None and self.fields:
            hit = getattr(self, "_midx", None)
            if hit is None or hit[0] is not mindex:
                idx = [mindex.get(f) for f in self.fields]
                hit = self._midx = (mindex, None if None in idx else np.asarray(idx, dtype=np.intp))
            if hit[1] is not None:
                return M[:, hit[1]]  # every referenced field is an input column: one gather
        X = np.empty((n, k), dtype=np.float64)
        if not self.fields:
            X[:] = 0.0
        for j, name in enumerate(self.fields):
            X[:, j] = cols.get(name)
        return X

    def leaves(self, X: np.ndarray) -> np.ndarray:
        """``int32 [T, n]`` scoring node of every row in every tree (local to the tree), -1 = null."""
        from ..native import fastpath

        fp = fastpath()
        X = np.ascontiguousarray(X, dtype=np.float64)
        ni, nd, kids, pi, pd, ai, ad, roots, modes, _ = self.arrays()
        out = np.empty((self.n_trees, X.shape[0]), dtype=np.int32)
        fp.forest_leaves(ni, nd, kids, pi, pd, ai, ad, roots, modes, X, X.shape[1], out, self.compiled())
        return out

    def values(self, X: np.ndarray) -> np.ndarray:
        """``float64 [n, T]`` leaf value of every row in every tree (NaN where the walk is null)."""
        from ..native import fastpath

        fp = fastpath()
        X = np.ascontiguousarray(X, dtype=np.float64)
        ni, nd, kids, pi, pd, ai, ad, roots, modes, lv = self.arrays()
        if lv.shape[0] != nd.shape[0]:
            raise ValueError("values() needs a leaf value for every node of every tree")
        out = np.empty((X.shape[0], self.n_trees), dtype=np.float64)
        fp.forest_values(ni, nd, kids, pi, pd, ai, ad, roots, modes, X, X.shape[1], lv, out, self.compiled())
        return out


    def sums(self, X: np.ndarray, weights: Optional[np.ndarray] = None) -> np.ndarray:
        """``float64 [n]``: per row, numpy's pairwise sum over the trees (in tree order) of the leaf
        value (times ``weights[t]``) -- bit-identical to ``np.sum(V * W, axis=1)`` of the
        :meth:`values` matrix; NaN where any tree is null."""
        from ..native import fastpath

        fp = fastpath()
        X = np.ascontiguousarray(X, dtype=np.float64)
        ni, nd, kids, pi, pd, ai, ad, roots, modes, lv = self.arrays()
        if lv.shape[0] != nd.shape[0]:
            raise ValueError("sums() needs a leaf value for every node of every tree")
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        out = np.empty(X.shape[0], dtype=np.float64)
        fp.forest_sums(ni, nd, kids, pi, pd, ai, ad, roots, modes, X, X.shape[1], lv, w, out, self.compiled())
        return out


    def votes(self, X: np.ndarray, cls: np.ndarray, weights: np.ndarray, C: int):
        """A (weighted) majority vote in one native call: ``(acc [n, C], wsum [n], count [n],
        anymiss [n])`` -- ``acc[r, cls[node]] += weights[t]`` for every tree whose scoring node has
        a class (``cls`` indexed by the program's global node ids, -1 = none), in tree order."""
        from ..native import fastpath

        fp = fastpath()
        X = np.ascontiguousarray(X, dtype=np.float64)
        ni, nd, kids, pi, pd, ai, ad, roots, modes, _ = self.arrays()
        n = X.shape[0]
        acc = np.empty((n, C), dtype=np.float64)
        wsum = np.empty(n, dtype=np.float64)
        count = np.empty(n, dtype=np.int32)
        miss = np.empty(n, dtype=np.uint8)
        fp.forest_votes(ni, nd, kids, pi, pd, ai, ad, roots, modes, X, X.shape[1],
                        np.ascontiguousarray(cls, dtype=np.int32), np.ascontiguousarray(weights, dtype=np.float64),
                        int(C), acc, wsum, count, miss, self.compiled())
        return acc, wsum, count, miss.astype(bool)


def native_available() -> bool:
    from ..native import fastpath

    fp = fastpath()
    return fp is not None and hasattr(fp, "forest_leaves")


def tree_program(ev) -> Optional[ForestProgram]:
    """One tree's program, or None (numpy walk)."""
    if not native_available():
        return None
    prog = ForestProgram(ev.schema)
    return prog if prog.add(ev) else None


def forest_program(evs: Sequence, leafvals: Sequence[np.ndarray]) -> Optional[ForestProgram]:
    """All of ``evs`` in one program with per-node leaf values, or None if any tree is not native."""
    if not native_available() or not evs:
        return None
    prog = ForestProgram(evs[0].schema)
    for ev, lv in zip(evs, leafvals):
        if not prog.add(ev, lv):
            return None
    return prog


__all__ = ["ForestProgram", "NotNative", "forest_program", "native_available", "tree_program"]
