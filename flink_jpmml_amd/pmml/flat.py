"""Flat (array) form of TreeModel bodies read by the native streaming scanner.

The reference parses every model into a JAXB object graph (`S/api/PmmlModel.scala:53-58`) and
advertises models of "several hundreds of MegaBytes" (`README.md:239-242`) — for tree ensembles
that is millions of ``<Node>`` elements. :func:`scan_document` runs the C++ scanner
(``native/csrc/pmml_scan.cpp``): one pass over the bytes, every TreeModel's node tree lands in the
arrays of a :class:`FlatTree`, and the remaining *skeleton* document (schemas, outputs, targets,
segment structure) is small enough for the regular parser.

Consumers that understand the flat form (tree evaluator set-up, binary lowering, field analysis)
read the arrays directly — no per-node Python objects. Anything else asks for ``TreeModel.root``
and gets an :class:`~flink_jpmml_amd.pmml.ir.Node` tree materialised once from the arrays (same
preorder numbering), so every code path sees the same model.
"""

from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import ir

P_NONE, P_TRUE, P_FALSE, P_SIMPLE, P_RAW = -1, 0, 1, 2, 3
OP_NAMES = ("equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual", "isMissing",
            "isNotMissing")

#: documents below this size are parsed the ordinary way (the scanner pays off on large ensembles)
SCAN_MIN_BYTES = 1 << 20


class FlatTree:
    """One TreeModel body: preorder node arrays (node 0 = root) plus the document's string table."""

    def __init__(self, arrays: Dict[str, np.ndarray], strings: Sequence[str], raw: Dict[int, bytes]):
        self.a = arrays
        self.strings = strings
        self.raw = raw  # node -> source bytes of a SimpleSetPredicate / CompoundPredicate
        n = len(arrays["parent"])
        self.n = n
        par = arrays["parent"]
        # children in document order (CSR): preorder => a stable sort by parent keeps sibling order
        order = np.argsort(par[1:], kind="stable") + 1
        counts = np.bincount(par[1:], minlength=n) if n > 1 else np.zeros(n, dtype=np.int64)
        self.child_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(counts, out=self.child_ptr[1:])
        self.child_idx = order.astype(np.int64)
        self.n_children = counts.astype(np.int64)
        self._lock = threading.Lock()
        self._root: Optional[ir.Node] = None
        # raw predicate spans parse now, so a malformed one fails the load like on the DOM path
        self.raw_pred: Dict[int, ir.Predicate] = {k: _parse_raw(v) for k, v in raw.items()}

    # ------------------------------------------------------------------ helpers
    def s(self, k: int) -> Optional[str]:
        return None if k < 0 else self.strings[k]

    def child(self, k: np.ndarray, pos: int) -> np.ndarray:
        """The ``pos``-th child of each node in ``k`` (callers know it exists)."""
        return self.child_idx[self.child_ptr[k] + pos]

    @property
    def max_depth(self) -> int:
        return int(self.a["depth"].max()) if self.n else 0

    def field_names(self) -> List[str]:
        """Fields the node predicates read (document order, unique), raw predicates included."""
        seen: Dict[str, None] = {}
        pf = self.a["pred_field"]
        ks = pf[(self.a["pred_kind"] == P_SIMPLE)]
        _, first = np.unique(ks, return_index=True)
        for k in ks[np.sort(first)]:
            seen.setdefault(self.strings[int(k)], None)
        for node in sorted(self.raw):
            from ..runtime.derive import _pred_fields

            _pred_fields(self.predicate(node), lambda f: seen.setdefault(f, None) if f is not None else None)
        return list(seen)

    def predicate(self, k: int) -> ir.Predicate:
        a = self.a
        kind = int(a["pred_kind"][k])
        if kind == P_TRUE:
            return ir.TruePredicate()
        if kind == P_FALSE:
            return ir.FalsePredicate()
        if kind == P_SIMPLE:
            return ir.SimplePredicate(self.strings[int(a["pred_field"][k])], OP_NAMES[int(a["pred_op"][k])],
                                      self.s(int(a["pred_value_s"][k])))
        if kind == P_RAW:
            return self.raw_pred[k]
        from ..api.exceptions import PmmlParseError

        raise PmmlParseError("<Node> has no predicate")

    # ------------------------------------------------------------------ materialisation
    def materialize(self) -> ir.Node:
        """The equivalent :class:`ir.Node` tree (built once; preorder numbering = array index)."""
        with self._lock:
            if self._root is not None:
                return self._root
            from ..utils.metrics import METRICS

            METRICS.inc("pmml.flat_materialized_nodes", self.n)
            a = self.a
            nodes: List[ir.Node] = []
            dist_node = a["dist_node"]
            dists: Dict[int, List[ir.ScoreDistribution]] = {}
            for j in range(len(dist_node)):
                p = float(a["dist_prob"][j])
                c = float(a["dist_conf"][j])
                dists.setdefault(int(dist_node[j]), []).append(ir.ScoreDistribution(
                    self.strings[int(a["dist_value_s"][j])], float(a["dist_count"][j]),
                    None if np.isnan(p) else p, None if np.isnan(c) else c))
            id_s, score_s, def_s, rc = a["id_s"], a["score_s"], a["default_s"], a["record_count"]
            for k in range(self.n):
                r = float(rc[k])
                nodes.append(ir.Node(id=self.s(int(id_s[k])), score=self.s(int(score_s[k])),
                                     predicate=self.predicate(k), record_count=None if np.isnan(r) else r,
                                     default_child=self.s(int(def_s[k])), distributions=dists.get(k, [])))
            par = a["parent"]
            for k in range(1, self.n):
                nodes[int(par[k])].children.append(nodes[k])
            self._root = nodes[0]
            return self._root


def _parse_raw(snippet: bytes) -> ir.Predicate:
    import xml.etree.ElementTree as ET

    from ..api.exceptions import PmmlParseError
    from .parser import _parse_predicate

    try:
        el = ET.fromstring(_with_ns(snippet))
        if el.tag.rsplit("}", 1)[-1] == "FjaWrap":
            el = el[0]
        return _parse_predicate(el)
    except ET.ParseError as e:
        raise PmmlParseError(f"malformed PMML XML in a tree predicate: {e}") from e
    except (ValueError, TypeError) as e:
        if isinstance(e, PmmlParseError):
            raise
        raise PmmlParseError(f"malformed PMML content in a tree predicate: {e}") from e


def _with_ns(snippet: bytes) -> bytes:
    """A raw predicate cut out of the document: wrap it so namespace prefixes / the default
    namespace parse (the parser only looks at local names)."""
    if b":" in snippet.split(b">", 1)[0].split(b" ", 1)[0]:
        prefix = snippet[1:snippet.index(b":")]
        return b"<FjaWrap xmlns:" + prefix + b'="http://www.dmg.org/PMML-4_4">' + snippet + b"</FjaWrap>"
    return snippet


def _py_float(s: str) -> float:
    try:
        return float(s)
    except ValueError:
        return float("nan")


def scan_document(data: bytes):
    """``(skeleton_bytes, [FlatTree])`` for a large document, or ``None`` (small document, no
    trees, scanner unavailable, or markup it does not represent: parse the ordinary way)."""
    if len(data) < SCAN_MIN_BYTES:
        return None
    from ..native import fastpath

    fp = fastpath()
    if fp is None:
        return None
    res = fp.scan_trees(data)
    if res is None:
        return None
    skeleton, trees, strings = res
    # the scanner reads numbers from ASCII strings only; Python's float() also takes Unicode digits
    # and white space, so non-ASCII scores / split values are settled here (DOM path: float(s))
    wide = [k for k, s in enumerate(strings) if not s.isascii()]
    if wide:
        num = np.full(len(strings) + 1, np.nan)
        for k in wide:
            num[k] = _py_float(strings[k])
        wide_a = np.zeros(len(strings) + 1, dtype=bool)
        wide_a[wide] = True
        for arrays in trees:
            for s_key, d_key in (("score_s", "score_d"), ("pred_value_s", "pred_value_d")):
                sk = arrays[s_key]
                m = wide_a[sk]  # index -1 (absent) hits the trailing False
                if m.any():
                    arrays[d_key][m] = num[sk[m]]
    flats = []
    for arrays in trees:
        raw = {}
        rs, re_ = arrays["raw_start"], arrays["raw_end"]
        for k in np.nonzero(rs >= 0)[0].tolist():
            raw[k] = bytes(data[int(rs[k]):int(re_[k])])
        flats.append(FlatTree(arrays, strings, raw))
    return skeleton, flats


__all__ = ["FlatTree", "SCAN_MIN_BYTES", "scan_document"]
