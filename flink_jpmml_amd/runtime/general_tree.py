"""GENERAL tree layout: node tables + predicate programs for ``tree.hip::tree_general_kernel``.

The branch-free PERFECT and POINTER layouts need binary ``x OP t`` splits. Every other PMML
TreeModel shape — multiway splits, ``SimpleSetPredicate``, ``CompoundPredicate`` (and / or / xor /
surrogate, the R ``rpart`` export), ``lastPrediction`` / ``nullPrediction`` / ``defaultChild`` /
``none`` missing strategies, ``returnLastPrediction``, scores on internal nodes — lowers here.
JPMML evaluates these by walking the object graph per record (`S/api/PmmlModel.scala:159-160`);
the kernel walks the same graph per lane, the semantics following the float64 oracle
:meth:`flink_jpmml_amd.models.tree.TreeEvaluator.leaf_index` exactly.

Predicates compile to postfix programs over three-valued logic. Comparisons against a constant
``t`` are made exact for fp32 inputs the same way as the binary layouts (directional rounding to a
``x >= T`` test, see :func:`flink_jpmml_amd.runtime.plans.canonical_threshold`); an equality with a
constant that no fp32 value can equal is compiled to "never equal".
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..models.tree import TreeEvaluator
from ..pmml import ir
from .plans import NotLowerable, _ceil32, _floor32, _next_up32

P_END, P_TRUE, P_FALSE, P_GE, P_EQ, P_ISMISS, P_NOTMISS, P_SET, P_AND, P_OR, P_XOR, P_SURR = range(12)
_COMPOUND = {"and": P_AND, "or": P_OR, "xor": P_XOR, "surrogate": P_SURR}
STRATEGY = {"none": 0, "lastPrediction": 1, "nullPrediction": 2, "defaultChild": 3, "weightedConfidence": 4,
            "aggregateNodes": 5}
MIX_STRATEGIES = ("weightedConfidence", "aggregateNodes")
MAX_STACK = 32  # 2-bit entries in the kernel's 64-bit stack
MIX_STACK = 64  # the mixture walk's explicit DFS stack (tree.hip::gen_mixture)


@dataclass
class GeneralTree:
    """Duck-types :class:`~flink_jpmml_amd.models.tree.BinaryTree` for the ensemble specs: per-node
    (``ev.nodes`` order) ``leaf_value`` (value or class index, NaN = no score) and ``leaf_probs``."""

    ev: TreeEvaluator
    field_index: Dict[str, int]
    leaf_value: np.ndarray
    leaf_probs: Optional[np.ndarray]
    has_score: np.ndarray
    depth: int
    null_missing: bool = True  # may yield no prediction (checked against skipSegment)
    # weightedConfidence / aggregateNodes: the sibling mixture a row takes at its first UNKNOWN
    # child (models/tree.py::_mixture) -- per node its class mass (tree category order) and its
    # weight as a child (recordCount / parent recordCount, or 1)
    mix_mass: Optional[np.ndarray] = None
    mix_w: Optional[np.ndarray] = None
    mix_vote: bool = False  # set by the ensemble lowering: this tree votes (majority) ...
    mix_weight: float = 1.0  # ... or averages its probabilities, with this segment weight
    mix_remap: Optional[np.ndarray] = None  # tree category -> accumulator slot
    value_col: Optional[np.ndarray] = None  # per node: kernel input column added to the leaf (or -1)


def lower_general_tree(ev: TreeEvaluator, field_index: Dict[str, int]) -> GeneralTree:
    if getattr(field_index, "folds", None):
        raise NotLowerable("folded derived fields need the binary tree lowering")
    tm = ev.tree
    if tm.missing_value_strategy not in STRATEGY:
        raise NotLowerable(f"missingValueStrategy {tm.missing_value_strategy!r} is host-only")
    classification = ev.kind == "classification"
    value = ev.node_label.copy() if classification else ev.node_value.copy()
    probs = ev.node_probs.copy() if classification else None
    depth = 0
    bound = 0  # worst-case DFS stack of the mixture walk: 1 + sum over a path of (children - 1)
    stack = [(tm.root, 0, 1)]
    while stack:
        nd, d, b = stack.pop()
        depth = max(depth, d)
        bound = max(bound, b)
        stack.extend((c, d + 1, b + max(0, len(nd.children) - 1)) for c in nd.children)
    gt = GeneralTree(ev, field_index, value, probs, ~np.isnan(value), depth)
    vf = getattr(ev, "value_fields", None)
    if vf:  # complex scorecard leaves: the score is a (derived) input column of the kernel
        if classification:  # pragma: no cover - only the regression scorecard rewrite sets them
            raise NotLowerable("per-record leaf values on a classification tree")
        col = np.full(len(ev.nodes), -1, dtype=np.int32)
        for i, name in vf.items():
            if name not in field_index:
                raise NotLowerable(f"leaf value field {name!r} is not a kernel input")
            col[i] = field_index[name]
        gt.value_col = col
    if tm.missing_value_strategy in MIX_STRATEGIES:
        if not classification:  # pragma: no cover - TreeEvaluator refuses it at load
            raise NotLowerable("weightedConfidence / aggregateNodes need a classification tree")
        if bound > MIX_STACK:
            raise NotLowerable(f"sibling mixture needs a {bound}-entry stack > {MIX_STACK}")
        nodes = ev.nodes
        gt.mix_mass = np.stack([ev._node_mass(i) for i in range(len(nodes))]).astype(np.float64)
        w = np.ones(len(nodes))
        if tm.missing_value_strategy == "weightedConfidence":
            index = ev._index
            for nd in nodes:
                pn = nd.record_count
                for c in nd.children:
                    cn = c.record_count
                    w[index[id(c)]] = (cn / pn) if cn is not None and pn else 1.0
        gt.mix_w = w
    return gt


class _PredCompiler:
    def __init__(self, schema, field_index: Dict[str, int]):
        self.schema = schema
        self.field_index = field_index
        self.code: List[tuple] = []
        self.pool: List[float] = []
        self.depth = 0
        self.max_depth = 0

    def _push(self, ins: tuple, pops: int = 0) -> None:
        self.code.append(ins)
        self.depth += 1 - pops
        self.max_depth = max(self.max_depth, self.depth)

    def _field(self, name: str) -> int:
        f = self.field_index.get(name)
        if f is None:
            raise NotLowerable(f"predicate on field {name!r} that is not a kernel input")
        return f

    def compile(self, p: ir.Predicate) -> int:
        off = len(self.code)
        self.depth = 0
        self._emit(p)
        self.code.append((P_END, 0, 0, 0))
        if self.max_depth > MAX_STACK:
            raise NotLowerable(f"predicate nests {self.max_depth} deep > {MAX_STACK}")
        return off

    def _emit(self, p: ir.Predicate) -> None:
        if isinstance(p, ir.TruePredicate):
            self._push((P_TRUE, 0, 0, 0))
        elif isinstance(p, ir.FalsePredicate):
            self._push((P_FALSE, 0, 0, 0))
        elif isinstance(p, ir.SimplePredicate):
            f = self._field(p.field)
            op = p.operator
            if op == "isMissing":
                self._push((P_ISMISS, f, 0, 0))
                return
            if op == "isNotMissing":
                self._push((P_NOTMISS, f, 0, 0))
                return
            v = float(self.schema.lookup(p.field, p.value))
            if op in ("lessThan", "greaterOrEqual"):  # x < v <=> not (x >= ceil32(v))
                T, neg = _ceil32(v), op == "lessThan"
                self._push((P_GE | (int(neg) << 8), f, 0, _bits(T)))
            elif op in ("lessOrEqual", "greaterThan"):  # x > v <=> x >= nextup(floor32(v))
                T, neg = _next_up32(_floor32(v)), op == "lessOrEqual"
                self._push((P_GE | (int(neg) << 8), f, 0, _bits(T)))
            elif op in ("equal", "notEqual"):
                T = float(np.float32(v)) if float(np.float32(v)) == v else float("nan")  # nan: never equal
                self._push((P_EQ | (int(op == "notEqual") << 8), f, 0, _bits(T)))
            else:
                raise NotLowerable(f"SimplePredicate operator {op!r}")
        elif isinstance(p, ir.SimpleSetPredicate):
            f = self._field(p.field)
            vals = [float(self.schema.lookup(p.field, v)) for v in p.values]
            vals = [v for v in vals if float(np.float32(v)) == v]  # fp32 inputs can only equal these
            off = len(self.pool)
            self.pool.extend(vals)
            self._push((P_SET | (int(p.boolean_operator == "isNotIn") << 8), f, off, len(vals)))
        elif isinstance(p, ir.CompoundPredicate):
            op = _COMPOUND.get(p.boolean_operator)
            if op is None or not p.predicates:
                raise NotLowerable(f"CompoundPredicate {p.boolean_operator!r}")
            for q in p.predicates:
                self._emit(q)
            self._push((op, len(p.predicates), 0, 0), pops=len(p.predicates))
        else:
            raise NotLowerable(f"predicate {type(p).__name__} is host-only")


def _bits(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.int32)[0])


def pack_general(trees: List[GeneralTree], weights: List[float], P: int, schema) -> dict:
    """Concatenate the trees' node tables into the kernel's arrays (``nodes`` int4, ``children``,
    ``preds`` int4, ``pool`` f32, ``trees`` int2, ``payload`` [nodes][P] f32) + ``max_steps``."""
    nodes: List[tuple] = []
    children: List[int] = []
    payload: List[np.ndarray] = []
    tree_tab: List[tuple] = []
    mix_tab: List[tuple] = []  # per tree {weight bits, vote, n classes, remap offset}
    mix_mass: List[np.ndarray] = []
    mix_w: List[np.ndarray] = []
    remap: List[int] = []
    any_mix = any(getattr(t, "mix_mass", None) is not None for t in trees)
    vcol: List[np.ndarray] = []
    any_vcol = any(getattr(t, "value_col", None) is not None for t in trees)
    pc: Optional[_PredCompiler] = None
    max_depth = 0
    for t, w in zip(trees, weights):
        ev = t.ev
        if pc is None:
            pc = _PredCompiler(schema, t.field_index)
        pc.field_index = t.field_index
        base = len(nodes)
        index = {id(nd): base + i for i, nd in enumerate(ev.nodes)}
        for i, nd in enumerate(ev.nodes):
            if len(nd.children) >= 1 << 16:
                raise NotLowerable("node with more than 65535 children")
            off = len(children)
            children.extend(index[id(c)] for c in nd.children)
            dflt = -1
            if nd.default_child is not None:
                for c in nd.children:
                    if c.id == nd.default_child:
                        dflt = index[id(c)]
                        break
            pred_off = pc.compile(nd.predicate)
            has = bool(t.has_score[i])
            nodes.append((off, len(nd.children) | (int(has) << 16), pred_off, dflt))
            if P > 1 and t.leaf_probs is not None:
                row = np.nan_to_num(np.asarray(t.leaf_probs[i], dtype=np.float64)[:P]) * w
            else:
                row = np.array([t.leaf_value[i] if has else 0.0]) * w
            payload.append(row)
        flags = STRATEGY[ev.tree.missing_value_strategy] | (
            (1 << 3) if ev.tree.no_true_child_strategy == "returnLastPrediction" else 0)
        tree_tab.append((base, flags))
        max_depth = max(max_depth, t.depth)
        if any_vcol:
            vc = getattr(t, "value_col", None)
            vcol.append(vc if vc is not None else np.full(len(ev.nodes), -1, dtype=np.int32))
        if any_mix:
            mm = getattr(t, "mix_mass", None)
            n = len(ev.nodes)
            if mm is None:
                mix_mass.append(np.zeros((n, P)))
                mix_w.append(np.ones(n))
                mix_tab.append((0, 0, 0, len(remap)))
            else:
                Ct = mm.shape[1]
                if Ct > P:
                    raise NotLowerable("tree has more categories than the ensemble's class slots")
                pad = np.zeros((n, P))
                pad[:, :Ct] = mm
                mix_mass.append(pad)
                mix_w.append(t.mix_w)
                rm = t.mix_remap if t.mix_remap is not None else np.arange(Ct)
                mix_tab.append((_bits(float(t.mix_weight)), int(bool(t.mix_vote)), Ct, len(remap)))
                remap.extend(int(x) for x in rm)
    return {
        "nodes": np.array(nodes, dtype=np.int64).astype(np.int32).reshape(-1, 4),
        "children": np.array(children or [0], dtype=np.int32),
        "preds": np.array(pc.code if pc else [(P_END, 0, 0, 0)], dtype=np.int64).astype(np.int32).reshape(-1, 4),
        "pool": np.array(pc.pool if pc and pc.pool else [0.0], dtype=np.float32),
        "trees": np.array(tree_tab, dtype=np.int32).reshape(-1, 2),
        "payload": np.stack(payload).astype(np.float32).reshape(len(nodes), -1),
        "max_steps": int(max_depth + 2),
        "mix_mass": np.concatenate(mix_mass).astype(np.float32).reshape(len(nodes), P) if any_mix else None,
        "mix_w": np.concatenate(mix_w).astype(np.float32) if any_mix else None,
        "mix_tab": np.array(mix_tab, dtype=np.int64).astype(np.int32).reshape(-1, 4) if any_mix else None,
        "remap": np.array(remap or [0], dtype=np.int32) if any_mix else None,
        "vcol": np.concatenate(vcol).astype(np.int32) if any_vcol else None,
    }


def emulate_general(packed: dict, X: np.ndarray, P: int, n_trees: int) -> np.ndarray:
    """numpy twin of the kernel walk (per row, per tree) -> ``[rows, P]`` accumulators, NaN for
    rows with a null tree (CPU tests)."""
    nodes, children, preds, pool = packed["nodes"], packed["children"], packed["preds"], packed["pool"]
    Xf = np.asarray(X, dtype=np.float32)
    out = np.zeros((len(Xf), P), dtype=np.float32)
    T = preds[:, 3].copy().view(np.float32)

    def ev(pc: int, x) -> int:
        st: List[int] = []
        while True:
            op, f, a, cnt = (int(v) for v in preds[pc])
            neg, op = (op >> 8) & 1, op & 0xFF
            if op == P_END:
                return st[-1]
            if op >= P_AND:
                vals = st[len(st) - f:]
                del st[len(st) - f:]
                if op == P_AND:
                    v = 0 if 0 in vals else (2 if 2 in vals else 1)
                elif op == P_OR:
                    v = 1 if 1 in vals else (2 if 2 in vals else 0)
                elif op == P_XOR:
                    v = 2 if 2 in vals else sum(1 for e in vals if e == 1) % 2
                else:
                    v = next((e for e in vals if e != 2), 2)
            elif op == P_TRUE:
                v = 1
            elif op == P_FALSE:
                v = 0
            else:
                xv = x[f]
                miss = bool(np.isnan(xv))
                if op == P_ISMISS:
                    v = int(miss)
                elif op == P_NOTMISS:
                    v = int(not miss)
                elif miss:
                    v = 2
                else:
                    if op == P_GE:
                        r = bool(xv >= T[pc])
                    elif op == P_EQ:
                        r = bool(xv == T[pc])
                    else:
                        r = bool(np.any(pool[a: a + cnt] == xv))
                    v = int(r) ^ neg
            st.append(v)
            pc += 1

    for r in range(len(Xf)):
        x = Xf[r]
        for t in range(n_trees):
            root, flags = (int(v) for v in packed["trees"][t])
            strat, ret_last = flags & 7, (flags >> 3) & 1
            node = root
            res = -1
            root_true = ev(int(nodes[node, 2]), x) == 1
            if root_true and strat >= 4:  # weightedConfidence / aggregateNodes
                res = _emulate_mixture(packed, ev, x, t, root, ret_last, P, out, r)
                if res is None:
                    continue
            if root_true:
                for _ in range(packed["max_steps"]):
                    off, nc, _, dflt = (int(v) for v in nodes[node])
                    nc &= 0xFFFF
                    if nc == 0:
                        res = node
                        break
                    nxt, stop = -1, False
                    for c in range(nc):
                        ch = int(children[off + c])
                        v = ev(int(nodes[ch, 2]), x)
                        if v == 2 and strat >= 4:  # pragma: no cover - mixture trees walk above
                            res, stop = -1, True
                            break
                        if v == 2 and strat != 0:
                            if strat == 1:
                                res, stop = node, True
                            elif strat == 2:
                                res, stop = -1, True
                            else:
                                nxt = dflt
                                if nxt < 0:
                                    res, stop = -1, True
                            break
                        if v == 1:
                            nxt = ch
                            break
                    if stop:
                        break
                    if nxt < 0:
                        res = node if ret_last else -1
                        break
                    node = nxt
            if res < 0 or not ((int(nodes[res, 1]) >> 16) & 1):
                out[r] = np.nan
            else:
                out[r] += packed["payload"][res]
                vc = packed.get("vcol")
                if vc is not None and int(vc[res]) >= 0:
                    out[r] += np.float32(x[int(vc[res])])
    return out


def _emulate_mixture(packed: dict, ev, x, t: int, root: int, ret_last: int, P: int, out: np.ndarray, r: int):
    """Twin of tree.hip::gen_walk + gen_mixture for a weightedConfidence / aggregateNodes tree: the
    ordinary walk while no predicate is UNKNOWN; at the first UNKNOWN the whole row restarts as the
    DFS sibling mixture. Adds the tree's payload to ``out[r]`` and returns None, or returns the
    scoring node / -1 of an ordinary walk for the caller to finish."""
    nodes, children = packed["nodes"], packed["children"]
    node = root
    for _ in range(packed["max_steps"]):
        off, nc, _, _ = (int(v) for v in nodes[node])
        nc &= 0xFFFF
        if nc == 0:
            return node
        nxt = -1
        unknown = False
        for c in range(nc):
            ch = int(children[off + c])
            v = ev(int(nodes[ch, 2]), x)
            if v == 2:
                unknown = True
                break
            if v == 1:
                nxt = ch
                break
        if unknown:
            break
        if nxt < 0:
            return node if ret_last else -1
        node = nxt
    else:  # pragma: no cover - max_steps bounds the depth
        return -1
    mm, mw, tab, remap = packed["mix_mass"], packed["mix_w"], packed["mix_tab"], packed["remap"]
    wbits, vote, Ct, roff = (int(v) for v in tab[t])
    w_tree = float(np.array([wbits], dtype=np.int32).view(np.float32)[0])
    mass = np.zeros(P, dtype=np.float32)
    stack = [(root, np.float32(1.0), False)]
    while stack:
        node, w, inside = stack.pop()
        off, nc, _, _ = (int(v) for v in nodes[node])
        nc &= 0xFFFF
        if nc == 0:
            mass += w * mm[node]
            continue
        k, vk = -1, 0
        vals = []
        for c in range(nc):
            ch = int(children[off + c])
            v = ev(int(nodes[ch, 2]), x)
            vals.append((ch, v))
            if k < 0 and v != 0:
                k, vk = c, v
        if k < 0:
            if ret_last:
                mass += w * mm[node]
            elif not inside:
                out[r] = np.nan
                return None
            continue
        if vk == 1:
            stack.append((vals[k][0], w, inside))
            continue
        for ch, v in reversed(vals[k:]):  # DFS order: child k first
            if v != 0:
                stack.append((ch, np.float32(w * mw[ch]), True))
    tot = float(mass[:Ct].sum())
    if not (np.isfinite(tot) and tot > 0):
        out[r] = np.nan
        return None
    if vote:
        lab = int(np.argmax(mass[:Ct]))
        out[r, remap[roff + lab]] += w_tree
    else:
        for c in range(Ct):
            out[r, remap[roff + c]] += np.float32(mass[c] / tot) * w_tree
    return None
