"""TreeModel: host oracle (general predicates) + binary-split lowering for the GPU.

Oracle semantics (PMML 4.x TreeModel): children are tried in document order, the first child
whose predicate is TRUE is followed. A predicate that is UNKNOWN (missing input) is handled by
``missingValueStrategy``:

* ``none`` — UNKNOWN counts as FALSE;
* ``lastPrediction`` — stop and return the current node's score;
* ``nullPrediction`` — no prediction (→ ``EmptyScore``);
* ``defaultChild`` — continue at the node's ``defaultChild``;
* ``weightedConfidence`` / ``aggregateNodes`` (classification) — at the first UNKNOWN child, the
  row is scored down that child and every sibling whose predicate is not FALSE (recursively);
  ``weightedConfidence`` sums the siblings' class confidences weighted by ``recordCount`` relative
  to the parent's, ``aggregateNodes`` sums the reached leaves' ScoreDistribution record counts; the
  winner is the largest class (probabilities: the normalised sum). Host-only (the device lowerings
  reject both strategies); parity unpinned — the PMML 4.4 text, no JPMML here.

When no child is TRUE, ``noTrueChildStrategy`` decides: ``returnNullPrediction`` (default) or
``returnLastPrediction``.

The oracle walks the tree breadth-first over *row subsets* with numpy, so a whole batch is
evaluated with O(nodes) vector operations.

:func:`lower_binary_tree` recognises the binary split form emitted by XGBoost / LightGBM /
scikit-learn exporters (two children: ``field OP threshold`` and its complement or ``True``) and
produces the (feature, threshold, op, default-direction, leaf) arrays of
:mod:`flink_jpmml_amd.runtime.plans` for the HIP traversal kernel.
"""

from __future__ import annotations

from collections.abc import Sequence
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema, eval_predicate
from .base import ModelEvaluator, ModelResult


class _RowView:
    __slots__ = ("cols", "rows", "n", "schema")

    def __init__(self, cols: Columns, rows: np.ndarray):
        self.cols = cols
        self.rows = rows
        self.n = int(len(rows))
        self.schema = cols.schema

    def get(self, name: str) -> np.ndarray:
        return self.cols.get(name)[self.rows]


class EntityLabels(Sequence):
    """Per-row ``entityId`` of the scoring node (None for a null prediction), materialised only
    when an output asks for it (a list comprehension per tree and batch otherwise dominated the
    host scoring of large ensembles)."""

    def __init__(self, ev: "TreeEvaluator", leaf: np.ndarray):
        self._ev = ev
        self._leaf = leaf
        self._list: Optional[List[Optional[str]]] = None

    def _materialise(self) -> List[Optional[str]]:
        if self._list is None:
            ids = [nd.id for nd in self._ev.nodes]
            self._list = [ids[i] if i >= 0 else None for i in self._leaf.tolist()]
        return self._list

    def __len__(self) -> int:
        return int(self._leaf.shape[0])

    def __getitem__(self, i):
        return self._materialise()[i]

    def __iter__(self):
        return iter(self._materialise())


class TreeEvaluator(ModelEvaluator):
    def __init__(self, model: ir.TreeModel, schema: FieldSchema):
        super().__init__(model, schema)
        self.tree = model
        if model.missing_value_strategy in ("weightedConfidence", "aggregateNodes") and \
                model.function_name != "classification":
            raise UnsupportedFeatureException(f"missingValueStrategy {model.missing_value_strategy!r} "
                                              "needs a classification TreeModel")
        self._nodes: Optional[List[ir.Node]] = None
        self._index_map: Optional[Dict[int, int]] = None
        if model.flat is not None:
            self._init_flat(model.flat)
            return
        self._build_node_list()
        if self.kind == "classification":
            cats = self.classification_categories()
            seen = set(cats)
            for nd in self.nodes:
                for s in [nd.score] + [d.value for d in nd.distributions]:
                    if s is not None and s not in seen:
                        cats.append(s)
                        seen.add(s)
            self.categories = cats
            C = len(cats)
            self.node_probs = np.zeros((len(self.nodes), C))
            self.node_label = np.full(len(self.nodes), NAN)
            for i, nd in enumerate(self.nodes):
                if nd.score is not None:
                    self.node_label[i] = cats.index(nd.score)
                if nd.distributions:
                    tot = sum(d.record_count for d in nd.distributions)
                    for d in nd.distributions:
                        p = d.probability if d.probability is not None else (d.record_count / tot if tot else 0.0)
                        self.node_probs[i, cats.index(d.value)] = p
                elif nd.score is not None:
                    self.node_probs[i, cats.index(nd.score)] = 1.0
        else:
            self.categories = None
            self.node_value = np.array([_num(nd.score) for nd in self.nodes], dtype=np.float64)
        # leaves whose score is read per record from a field (complex scorecards)
        self.value_fields = {i: nd.value_field for i, nd in enumerate(self.nodes) if nd.value_field is not None}

    # -- node list (preorder, first child first): built from the IR, or materialised lazily from a
    #    flat body (pmml/flat.py) only when an object-level consumer needs it
    def _build_node_list(self) -> None:
        nodes: List[ir.Node] = []
        index: Dict[int, int] = {}
        stack = [self.tree.root]
        while stack:
            nd = stack.pop()
            index[id(nd)] = len(nodes)
            nodes.append(nd)
            stack.extend(reversed(nd.children))
        self._nodes, self._index_map = nodes, index

    @property
    def nodes(self) -> List[ir.Node]:
        if self._nodes is None:
            self._build_node_list()
        return self._nodes

    @property
    def _index(self) -> Dict[int, int]:
        if self._index_map is None:
            self._build_node_list()
        return self._index_map

    def _init_flat(self, ft) -> None:
        """Node tables straight from the flat arrays (same values as the object path)."""
        a = ft.a
        n = ft.n
        if self.kind != "classification":
            self.categories = None
            self.node_value = np.array(a["score_d"], dtype=np.float64)
            return
        cats = self.classification_categories()
        strings = ft.strings
        # categories beyond the declared ones, in first-appearance order over (score, distributions…)
        keys = np.concatenate([np.arange(n, dtype=np.int64) * 2, a["dist_node"].astype(np.int64) * 2 + 1])
        vals = np.concatenate([a["score_s"], a["dist_value_s"]]).astype(np.int64)
        order = np.argsort(keys, kind="stable")
        seq = vals[order]
        seq = seq[seq >= 0]
        uniq, first = np.unique(seq, return_index=True)
        seen = set(cats)
        for k in uniq[np.argsort(first)]:
            v = strings[int(k)]
            if v not in seen:
                cats.append(v)
                seen.add(v)
        self.categories = cats
        cat_of = {c: i for i, c in enumerate(cats)}
        code = np.full(len(strings) + 1, -1, dtype=np.int64)  # string index -> category (-1: none)
        for k in np.unique(np.concatenate([a["score_s"], a["dist_value_s"]])).tolist():
            if k >= 0:
                code[k] = cat_of[strings[k]]
        C = len(cats)
        sc = code[a["score_s"]]
        self.node_label = np.where(sc >= 0, sc, NAN).astype(np.float64)
        probs = np.zeros((n, C))
        has_score = sc >= 0
        probs[np.nonzero(has_score)[0], sc[has_score]] = 1.0
        dn = a["dist_node"].astype(np.int64)
        if dn.size:
            tot = np.bincount(dn, weights=a["dist_count"], minlength=n)
            p = np.where(np.isnan(a["dist_prob"]),
                         np.divide(a["dist_count"], tot[dn], out=np.zeros(dn.size), where=tot[dn] != 0),
                         a["dist_prob"])
            with_d = np.unique(dn)
            probs[with_d] = 0.0  # distributions replace the score's one-hot
            probs[dn, code[a["dist_value_s"]]] = p
        self.node_probs = probs

    def native_program(self):
        """This tree's :class:`~flink_jpmml_amd.models.native_tree.ForestProgram` (built once), or
        None when the tree keeps the numpy walk."""
        prog = getattr(self, "_native", False)
        if prog is False:
            from .native_tree import tree_program

            prog = self._native = tree_program(self)
        return prog

    def leaf_index(self, cols: Columns) -> np.ndarray:
        """Index (into ``self.nodes``) of the scoring node per row; -1 = null prediction. Runs the
        native walker (``models/native_tree.py``, the same decisions in C++) when the tree has a
        program and every field it references can be prepared, else the numpy walk below."""
        prog = self.native_program()
        if prog is not None and cols.n:
            try:
                X = prog.matrix(cols)
            except Exception:  # noqa: BLE001 - e.g. a field only unreachable nodes reference
                X = None
            if X is not None:
                return prog.leaves(X)[0].astype(np.int64)
        return self.leaf_index_numpy(cols)

    def leaf_index_numpy(self, cols: Columns) -> np.ndarray:
        """The numpy-mask walk (the semantic reference of the native walker)."""
        n = cols.n
        out = np.full(n, -1, dtype=np.int64)
        strat = self.tree.missing_value_strategy
        no_true = self.tree.no_true_child_strategy
        work: List[Tuple[ir.Node, np.ndarray]] = [(self.tree.root, np.arange(n))]
        # the root's own predicate (normally True) selects the rows that reach it
        root_t, _ = eval_predicate(self.tree.root.predicate, cols)
        work = [(self.tree.root, np.nonzero(root_t)[0])]
        while work:
            node, rows = work.pop()
            if rows.size == 0:
                continue
            me = self._index[id(node)]
            if not node.children:
                out[rows] = me
                continue
            remaining = rows
            by_id = {c.id: c for c in node.children}
            for child in node.children:
                if remaining.size == 0:
                    break
                view = _RowView(cols, remaining)
                t, u = eval_predicate(child.predicate, view)
                if u.any() and strat != "none":
                    urows = remaining[u]
                    if strat == "lastPrediction":
                        out[urows] = me
                    elif strat == "defaultChild":
                        dc = by_id.get(node.default_child)
                        if dc is not None:
                            work.append((dc, urows))
                    # nullPrediction: stays -1
                    keep = ~u
                    t = t[keep]
                    remaining = remaining[keep]
                if t.any():
                    work.append((child, remaining[t]))
                    remaining = remaining[~t]
            if remaining.size and no_true == "returnLastPrediction":
                out[remaining] = me
        return out

    def _node_mass(self, i: int) -> np.ndarray:
        """Per-class mass a node contributes: ScoreDistribution record counts (aggregateNodes) or
        its class confidences (weightedConfidence)."""
        nd = self.nodes[i]
        if self.tree.missing_value_strategy == "aggregateNodes":
            v = np.zeros(len(self.categories))
            for d in nd.distributions:
                v[self.categories.index(d.value)] += d.record_count
            if not nd.distributions and nd.score is not None:
                v[self.categories.index(nd.score)] = nd.record_count if nd.record_count else 1.0
            return v
        return self.node_probs[i]

    def _mixture(self, node: ir.Node, cols, rows: np.ndarray) -> np.ndarray:
        """``[len(rows), C]`` class mass of the rows that reached ``node`` (NaN row: no prediction)."""
        C = len(self.categories)
        me = self._index[id(node)]
        out = np.full((rows.size, C), NAN)
        if rows.size == 0:
            return out
        if not node.children:
            out[:] = self._node_mass(me)
            return out
        view = _RowView(cols, rows)
        evals = [eval_predicate(c.predicate, view) for c in node.children]
        todo = np.ones(rows.size, dtype=bool)
        for k, child in enumerate(node.children):
            t, u = evals[k]
            go = todo & t & ~u
            if go.any():  # TRUE before any UNKNOWN: the ordinary walk
                out[go] = self._mixture(child, cols, rows[go])
            unk = todo & u
            if unk.any():  # first UNKNOWN: this child and every later sibling not FALSE
                acc = np.zeros((int(unk.sum()), C))
                parent_n = node.record_count
                for j in range(k, len(node.children)):
                    tj, uj = evals[j]
                    sel = (tj | uj)[unk]
                    if not sel.any():
                        continue
                    sub = self._mixture(node.children[j], cols, rows[unk][sel])
                    w = 1.0
                    if self.tree.missing_value_strategy == "weightedConfidence":
                        cn = node.children[j].record_count
                        w = (cn / parent_n) if cn is not None and parent_n else 1.0
                    acc[sel] += np.nan_to_num(sub, nan=0.0) * w
                out[unk] = acc
            todo &= ~(t | u)
        if todo.any() and self.tree.no_true_child_strategy == "returnLastPrediction":
            out[todo] = self._node_mass(me)
        return out

    def _mix_rows(self, res: ModelResult, cols: Columns, leaf: np.ndarray) -> ModelResult:
        """Rows the ordinary walk left without a node (an UNKNOWN on the way, or no TRUE child):
        the recursive sibling mixture; rows that never met an UNKNOWN keep their leaf's result."""
        root_t, _ = eval_predicate(self.tree.root.predicate, cols)
        rows = np.nonzero(root_t & (leaf < 0))[0]
        if rows.size == 0:
            return res
        mass = self._mixture(self.tree.root, cols, rows)
        tot = mass.sum(axis=1)
        ok = np.isfinite(tot) & (tot > 0)
        with np.errstate(invalid="ignore", divide="ignore"):
            probs = np.where(ok[:, None], mass / np.where(ok, tot, 1.0)[:, None], NAN)
        lab = np.where(ok, np.argmax(np.nan_to_num(mass, nan=-np.inf), axis=1), 0).astype(np.float64)
        res.value[rows] = np.where(ok, lab, NAN)
        res.valid[rows] = ok
        res.probs[rows] = probs
        return res

    def _evaluate(self, cols: Columns) -> ModelResult:
        leaf = self.leaf_index(cols)
        ok = leaf >= 0
        safe = np.where(ok, leaf, 0)
        ent = EntityLabels(self, leaf)
        if self.kind == "classification":
            lab = np.where(ok, self.node_label[safe], NAN)
            ok = ok & ~np.isnan(lab)
            probs = np.where(ok[:, None], self.node_probs[safe], NAN)
            res = ModelResult("classification", np.where(ok, lab, NAN), ok, categories=self.categories, probs=probs)
            if self.tree.missing_value_strategy in ("weightedConfidence", "aggregateNodes"):
                res = self._mix_rows(res, cols, leaf)
        else:
            val = np.where(ok, self.node_value[safe], NAN)
            for i, name in getattr(self, "value_fields", {}).items():
                m = leaf == i
                if m.any():
                    val[m] = cols.get(name)[m]
            ok = ok & ~np.isnan(val)
            res = ModelResult("regression", val, ok)
        res.extra["entity_labels"] = ent
        res.extra["leaf"] = leaf
        return res


def _num(s: Optional[str]) -> float:
    if s is None:
        return NAN
    try:
        return float(s)
    except ValueError:
        return NAN


# --------------------------------------------------------------------------- lowering

# comparison opcodes understood by the HIP kernel: go LEFT when  x OP threshold
OP_LT, OP_LE, OP_GT, OP_GE = 0, 1, 2, 3
_OPS = {"lessThan": OP_LT, "lessOrEqual": OP_LE, "greaterThan": OP_GT, "greaterOrEqual": OP_GE}
_NEG = {"lessThan": "greaterOrEqual", "lessOrEqual": "greaterThan", "greaterThan": "lessOrEqual",
        "greaterOrEqual": "lessThan"}


@dataclass
class BinaryTree:
    """Pointer-form binary tree: arrays indexed by node id (0 = root)."""

    feature: np.ndarray  # int32, -1 for leaves
    threshold: np.ndarray  # float64
    op: np.ndarray  # int8, go-left condition
    default_left: np.ndarray  # bool: where a missing value goes
    left: np.ndarray  # int32
    right: np.ndarray  # int32
    leaf_value: np.ndarray  # float64 (regression) / class index (classification)
    leaf_probs: Optional[np.ndarray]  # [nodes, C] or None
    depth: int
    null_missing: bool = False  # a missing value at any visited split -> null prediction


class NotBinary(Exception):
    pass


def membership_key(field: str, values) -> str:
    """Name of the synthetic 0/1 column "``field`` is one of ``values``" (derive program)."""
    return "__in__(" + field + "|" + "|".join(sorted(str(v) for v in values)) + ")"


def member_form(pa: ir.Predicate, pb: ir.Predicate):
    """``(field, values, first_child_is_member)`` when the two child predicates are a categorical
    binary split — ``isIn S`` / ``isNotIn S`` (LightGBM, sklearn2pmml) or ``== v`` / ``!= v``
    (R, KNIME) with the complement or ``True`` as second child — else None."""
    if isinstance(pa, ir.SimpleSetPredicate) and pa.boolean_operator in ("isIn", "isNotIn"):
        ok = isinstance(pb, ir.TruePredicate) or (
            isinstance(pb, ir.SimpleSetPredicate) and pb.field == pa.field
            and sorted(pb.values) == sorted(pa.values) and pb.boolean_operator != pa.boolean_operator)
        return (pa.field, tuple(pa.values), pa.boolean_operator == "isIn") if ok else None
    if isinstance(pa, ir.SimplePredicate) and pa.operator in ("equal", "notEqual") and pa.value is not None:
        neg = "notEqual" if pa.operator == "equal" else "equal"
        ok = isinstance(pb, ir.TruePredicate) or (
            isinstance(pb, ir.SimplePredicate) and pb.field == pa.field and pb.value == pa.value
            and pb.operator == neg)
        return (pa.field, (pa.value,), pa.operator == "equal") if ok else None
    return None


def _flat_member_candidates(ft) -> bool:
    """Whether a flat body has binary splits whose first child is a set or (in)equality
    predicate (the shapes :func:`member_form` turns into membership columns)."""
    from ..pmml.flat import P_RAW, P_SIMPLE

    internal = np.nonzero(ft.n_children == 2)[0]
    if internal.size == 0:
        return False
    ca = ft.child(internal, 0)
    kind, op = ft.a["pred_kind"][ca], ft.a["pred_op"][ca]
    return bool(np.any(kind == P_RAW) or np.any((kind == P_SIMPLE) & (op <= 1)))


def membership_fields(model: ir.Model) -> Dict[str, ir.DerivedField]:
    """Synthetic DerivedFields (MapValues lookups: member 1, non-member 0, missing -> missing) for
    every categorical binary split of the model's trees (nested segments included)."""
    out: Dict[str, ir.DerivedField] = {}

    def walk(m: ir.Model) -> None:
        if isinstance(m, ir.MiningModel):
            for seg in m.segments:
                walk(seg.model)
            return
        if not isinstance(m, ir.TreeModel):
            return
        if m.flat is not None and not _flat_member_candidates(m.flat):
            return  # no set / equality splits: nothing to add (no object materialisation)
        stack = [m.root]
        while stack:
            nd = stack.pop()
            stack.extend(nd.children)
            if len(nd.children) != 2:
                continue
            f = member_form(nd.children[0].predicate, nd.children[1].predicate)
            if f is None:
                continue
            name = membership_key(f[0], f[1])
            if name not in out:
                rows = [{"k": v, "o": "1"} for v in f[1]]
                expr = ir.MapValues(output_column="o", field_columns=[(f[0], "k")], rows=rows, default_value="0")
                out[name] = ir.DerivedField(name, "continuous", "double", expr)

    walk(model)
    return out


_FLAT_NUMERIC_OPS = {2: "lessThan", 3: "lessOrEqual", 4: "greaterThan", 5: "greaterOrEqual"}


def _lower_flat(ev: TreeEvaluator, ft, field_index: Dict[str, int]) -> Optional[BinaryTree]:
    """:func:`lower_binary_tree` on a flat body, vectorised (no per-node Python). Returns ``None``
    for shapes it leaves to the object path (categorical member splits, folded fields)."""
    from ..pmml.flat import P_RAW, P_SIMPLE, P_TRUE

    tm = ev.tree
    strat = tm.missing_value_strategy
    a = ft.a
    kind = a["pred_kind"]
    if kind[0] != P_TRUE:
        raise NotBinary("root predicate is not True")
    n = ft.n
    nch = ft.n_children
    internal = np.nonzero(nch > 0)[0]
    leaves = nch == 0
    if np.any(nch[internal] != 2):
        raise NotBinary("node does not have exactly two children")
    ca, cb = ft.child(internal, 0), ft.child(internal, 1)
    ka, kb = kind[ca], kind[cb]
    opa, opb = a["pred_op"][ca], a["pred_op"][cb]
    if np.any(ka == P_RAW) or np.any(kb == P_RAW) or np.any((ka == P_SIMPLE) & (opa <= 1)):
        return None  # SimpleSet / equality splits: membership columns (object path)
    folds = getattr(field_index, "folds", None) or {}
    if np.any(ka != P_SIMPLE) or np.any((opa < 2) | (opa > 5)):
        raise NotBinary("first child predicate is not a numeric comparison")
    fa = a["pred_field"][ca]
    uniq_f = np.unique(fa)
    fcol = np.full(len(ft.strings) + 1, -1, dtype=np.int32)
    for k in uniq_f.tolist():
        name = ft.strings[k]
        if name in folds:
            return None  # monotone derived fields fold per split value (object path)
        if name not in field_index or ev.schema.is_string(name):
            raise NotBinary("split on a non-input or string field")
        fcol[k] = field_index[name]
    neg = np.array([1, 0, 5, 4, 3, 2, 7, 6], dtype=np.int8)  # _NEG on operator codes
    comp = (kb == P_SIMPLE) & (a["pred_field"][cb] == fa) & (opb == neg[opa]) & \
        (a["pred_value_s"][cb] == a["pred_value_s"][ca])
    second_true = kb == P_TRUE
    if not np.all(second_true | comp):
        raise NotBinary("second child is not the complement of the first")
    t = a["pred_value_d"][ca]
    if np.any(np.isnan(t)) and np.any(np.isnan(t) & (a["pred_value_s"][ca] >= 0)):
        raise NotBinary("non-numeric split value")
    forms = set()
    if strat == "defaultChild":
        if np.any(a["default_s"][internal] < 0):
            raise NotBinary("defaultChild strategy without defaultChild attribute")
        dp = a["default_pos"][internal]
        if np.any((dp != 0) & (dp != 1)):
            raise NotBinary("defaultChild does not name a child")
        go_left = dp == 0
    elif strat == "nullPrediction":
        go_left = np.zeros(internal.size, dtype=bool)
    else:
        if second_true.any():
            forms.add("true")
        if (~second_true).any():
            if tm.no_true_child_strategy != "returnNullPrediction":
                raise NotBinary("missing value under returnLastPrediction needs internal-node scores")
            forms.add("complement")
        if len(forms) > 1:
            raise NotBinary("'none' strategy mixing True and complement second children")
        go_left = np.zeros(internal.size, dtype=bool)
    classification = ev.kind == "classification"
    leaf_idx = np.nonzero(leaves)[0]
    leafv = np.full(n, NAN)
    if classification:
        leafv[leaf_idx] = ev.node_label[leaf_idx]
    else:
        leafv[leaf_idx] = ev.node_value[leaf_idx]
    if np.any(np.isnan(leafv[leaf_idx])):
        raise NotBinary("leaf without score")
    feature = np.full(n, -1, dtype=np.int32)
    thr = np.zeros(n)
    op = np.zeros(n, dtype=np.int8)
    dleft = np.zeros(n, dtype=bool)
    left = np.full(n, -1, dtype=np.int32)
    right = np.full(n, -1, dtype=np.int32)
    feature[internal] = fcol[fa]
    thr[internal] = t
    code = np.zeros(8, dtype=np.int8)
    for k, name in _FLAT_NUMERIC_OPS.items():
        code[k] = _OPS[name]
    op[internal] = code[opa]
    dleft[internal] = go_left
    left[internal], right[internal] = ca, cb
    probs = None
    if classification:
        probs = np.zeros((n, len(ev.categories)))
        probs[leaf_idx] = ev.node_probs[leaf_idx]
    return BinaryTree(feature=feature, threshold=thr, op=op, default_left=dleft, left=left, right=right,
                      leaf_value=leafv, leaf_probs=probs, depth=int(a["depth"][leaves].max()) if n else 0,
                      null_missing=strat == "nullPrediction" or forms == {"complement"})


def lower_binary_tree(ev: TreeEvaluator, field_index: Dict[str, int]) -> BinaryTree:
    """Lower a TreeModel into pointer-form binary arrays, or raise :class:`NotBinary`.

    Accepted node shapes (all exporters we know of use one of them):

    * two children ``[x OP t, True]`` or ``[x OP t, x NEG(OP) t]``;
    * missing values: ``defaultChild`` strategy (per-node default); ``none`` strategy with a
      ``True`` second child (missing → right); ``nullPrediction`` — and ``none`` with complement
      children under ``returnNullPrediction`` — make the whole tree's prediction null on a
      missing split value (``null_missing``: the kernels poison the row). ``lastPrediction`` (and
      ``returnLastPrediction`` on a missing value) needs internal-node scores and raises
      :class:`NotBinary`.
    """
    tm = ev.tree
    strat = tm.missing_value_strategy
    if strat not in ("none", "defaultChild", "nullPrediction"):
        raise NotBinary(f"missingValueStrategy {strat}")
    if tm.flat is not None:
        bt = _lower_flat(ev, tm.flat, field_index)
        if bt is not None:
            return bt
    null_missing = strat == "nullPrediction"
    forms = set()  # 'none' strategy: second child True (missing -> right) or complement (-> null)
    if not isinstance(tm.root.predicate, ir.TruePredicate):
        raise NotBinary("root predicate is not True")
    feats: List[int] = []
    thr: List[float] = []
    ops: List[int] = []
    dleft: List[bool] = []
    lefts: List[int] = []
    rights: List[int] = []
    leafv: List[float] = []
    leafp: List[np.ndarray] = []
    classification = ev.kind == "classification"

    def new_node() -> int:
        feats.append(-1)
        thr.append(0.0)
        ops.append(0)
        dleft.append(False)
        lefts.append(-1)
        rights.append(-1)
        leafv.append(NAN)
        if classification:
            leafp.append(np.zeros(len(ev.categories)))
        return len(feats) - 1

    folds = getattr(field_index, "folds", None) or {}  # runtime/derive.py: monotone derived fields
    folded: Dict[str, List[int]] = {}
    max_depth = 0
    stack = [(tm.root, new_node(), 0)]
    while stack:
        node, k, depth = stack.pop()
        max_depth = max(max_depth, depth)
        i = ev._index[id(node)]
        if not node.children:
            if classification:
                leafv[k] = ev.node_label[i]
                leafp[k] = ev.node_probs[i]
            else:
                leafv[k] = ev.node_value[i]
            if np.isnan(leafv[k]):
                raise NotBinary("leaf without score")
            continue
        if len(node.children) != 2:
            raise NotBinary("node does not have exactly two children")
        a, b = node.children
        pa, pb = a.predicate, b.predicate
        member = member_form(pa, pb)
        if member is not None:
            # categorical split (set / equality): numeric split on its 0/1 membership column
            split_field = membership_key(member[0], member[1])
            if split_field not in field_index:
                raise NotBinary("categorical split without a membership column")
            split_t, split_op = 0.5, (OP_GE if member[2] else OP_LT)
        else:
            if not isinstance(pa, ir.SimplePredicate) or pa.operator not in _OPS:
                raise NotBinary("first child predicate is not a numeric comparison")
            if pa.field not in field_index or ev.schema.is_string(pa.field):
                raise NotBinary("split on a non-input or string field")
            if isinstance(pb, ir.TruePredicate):
                pass
            elif isinstance(pb, ir.SimplePredicate) and pb.field == pa.field and pb.operator == _NEG[pa.operator] \
                    and pb.value == pa.value:
                pass
            else:
                raise NotBinary("second child is not the complement of the first")
            split_field, split_t, split_op = pa.field, float(pa.value), _OPS[pa.operator]
        # missing-value direction
        if strat == "defaultChild":
            if node.default_child is None:
                raise NotBinary("defaultChild strategy without defaultChild attribute")
            go_left = node.default_child == a.id
            if not go_left and node.default_child != b.id:
                raise NotBinary("defaultChild does not name a child")
        elif strat == "nullPrediction":
            go_left = False  # never used: the prediction is null
        else:
            # 'none': UNKNOWN counts as FALSE -> a missing value fails the first predicate; the
            # second child is taken if it is True; a complement predicate is also UNKNOWN -> no
            # true child -> noTrueChildStrategy (null prediction lowers, last prediction does not)
            if isinstance(pb, ir.TruePredicate):
                forms.add("true")
            elif tm.no_true_child_strategy == "returnNullPrediction":
                forms.add("complement")
            else:
                raise NotBinary("missing value under returnLastPrediction needs internal-node scores")
            if len(forms) > 1:
                raise NotBinary("'none' strategy mixing True and complement second children")
            go_left = False
        if split_field in folds:
            folded.setdefault(split_field, []).append(k)
        feats[k] = field_index[split_field]
        thr[k] = split_t
        ops[k] = split_op
        dleft[k] = go_left
        la, lb = new_node(), new_node()
        lefts[k], rights[k] = la, lb
        stack.append((a, la, depth + 1))
        stack.append((b, lb, depth + 1))
    thr_a, ops_a = np.array(thr, dtype=np.float64), np.array(ops, dtype=np.int8)
    if folded:  # splits on a monotone derived field -> splits on its source input
        from ..runtime.derive import fold_splits

        for name, ks in folded.items():
            _, f, memo = folds[name]
            for k in ks:
                hit = memo.get((int(ops_a[k]), float(thr_a[k])))
                if hit is None:  # not pre-resolved (runtime/derive.py::_resolve_folds)
                    o, t = fold_splits(f, ops_a[k:k + 1], thr_a[k:k + 1])
                    hit = memo[(int(ops_a[k]), float(thr_a[k]))] = (int(o[0]), float(t[0]))
                ops_a[k], thr_a[k] = hit
    return BinaryTree(
        feature=np.array(feats, dtype=np.int32),
        threshold=thr_a,
        op=ops_a,
        default_left=np.array(dleft, dtype=bool),
        left=np.array(lefts, dtype=np.int32),
        right=np.array(rights, dtype=np.int32),
        leaf_value=np.array(leafv, dtype=np.float64),
        leaf_probs=np.stack(leafp) if classification else None,
        depth=max_depth,
        null_missing=null_missing or forms == {"complement"},
    )
