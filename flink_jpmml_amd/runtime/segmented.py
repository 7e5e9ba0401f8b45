"""MiningModel segmentations the fused tree kernel cannot express, on the device.

The fused ensemble kernels (:class:`~flink_jpmml_amd.runtime.plans.TreePlan`) cover ``sum`` /
``average`` / ``weightedAverage`` / majority votes over ``True`` segments of binary trees and the
model chains of XGBoost / LightGBM. Everything else a JPMML user can hand the reference
(`S/api/PmmlModel.scala:159-160` evaluates any segmentation JPMML supports) lowers here:

* ``multipleModelMethod`` ``selectFirst``, ``max``, ``min``, ``median``, ``weightedMedian`` and
  every supported method under **non-True segment predicates** (the segment participates only
  where its predicate is TRUE; three-valued logic, UNKNOWN does not select);
* classification ``average`` / ``weightedAverage`` / ``max`` / ``median`` over the segments'
  probability vectors (each segment plan writes its ``[n, C_i]`` probabilities through its fused
  epilogue; they are scattered into the ensemble's category order on the device);
* segments that are not binary trees: each segment is lowered by :func:`compile_plan` on its own
  (trees, linear models, neural networks, SVMs, nested ensembles — recursively).

Execution: every segment plan scores the (already prepared) input matrix on the caller's stream,
the segment predicates are evaluated with fp64 tensor ops on the same matrix (exact parity with
the oracle's float64 comparisons of the fp32 inputs), and the aggregation — the oracle's
``MiningEvaluator._select/_regress/_classify`` (`models/mining.py`) — runs as tensor ops. No host
round trip; the per-segment launches make this a slower path than the fused kernels, which is
why it is only taken when they refuse the model.

Inputs must be prepared (MiningField treatment applied once, as the oracle does at the top
level): :func:`compile_plan` puts a prepare-only derive pass in front when the model needs one.
"""

from __future__ import annotations

import contextlib
from typing import List, Optional

import numpy as np

from ..models.mining import MiningEvaluator
from ..pmml import ir
from .plans import (VAR_POINTER_COMPACT, VAR_POINTER_INLINE, VAR_POINTER_LDS, VAR_POINTER_RANK3, VAR_POINTER_REFILL,
                    VAR_POINTER_SUPER, DevicePlan, NotLowerable, _label_table,
                    apply_target_torch, target_post)

REGRESSION_METHODS = ("sum", "average", "weightedAverage", "max", "min", "median", "weightedMedian", "selectFirst")
PROB_METHODS = ("average", "weightedAverage", "max", "median")  # classification over segment probabilities
CLASSIFICATION_METHODS = ("majorityVote", "weightedMajorityVote", "selectFirst") + PROB_METHODS


class SubView:
    """One segment's model seen through its parent's (prepared) input columns."""

    fields_resolved = True
    prepared_inputs = True

    def __init__(self, parent, evaluator):
        self._p = parent
        self.evaluator = evaluator
        self.model = evaluator.model
        self.mining_fields = {}
        self.target_fields = list(parent.target_fields)

    def __getattr__(self, name):
        return getattr(self._p, name)


def segmentable(ev, compiled) -> Optional[str]:
    """None when :class:`SegmentedPlan` can lower ``ev``; else the reason."""
    if not isinstance(ev, MiningEvaluator):
        return "not a MiningModel"
    method = ev.method
    if ev.kind == "regression" and method not in REGRESSION_METHODS:
        return f"regression multipleModelMethod {method!r}"
    if ev.kind == "classification" and method not in CLASSIFICATION_METHODS:
        return f"classification multipleModelMethod {method!r}"
    if ev.kind not in ("regression", "classification"):
        return f"{ev.kind} segmentation"
    # MiningModel- and segment-level LocalTransformations are computed by the derive pass in front
    # of this plan (runtime/derive.py::collect_derived walks the segments): the segment plans and
    # predicates read them as columns of the augmented matrix
    for seg in ev.segments:
        why = _predicate_fields_ok(seg.predicate, compiled)
        if why:
            return why
    return None


def _predicate_fields_ok(p, compiled) -> Optional[str]:
    if isinstance(p, (ir.TruePredicate, ir.FalsePredicate)):
        return None
    if isinstance(p, (ir.SimplePredicate, ir.SimpleSetPredicate)):
        fi = getattr(compiled, "field_index", None) or {f: i for i, f in enumerate(compiled.active_fields)}
        return None if p.field in fi else f"segment predicate on non-input field {p.field!r}"
    if isinstance(p, ir.CompoundPredicate):
        if p.boolean_operator not in ("and", "or", "xor", "surrogate"):
            return f"CompoundPredicate {p.boolean_operator!r}"
        for q in p.predicates:
            why = _predicate_fields_ok(q, compiled)
            if why:
                return why
        return None
    return f"segment predicate {type(p).__name__}"


def compile_predicate(p, compiled):
    """A segment predicate as a picklable program with columns and categorical codes resolved:
    ``("T",)`` / ``("F",)`` / ``("S", col, op, value)`` / ``("M", col, isMissing)`` /
    ``("I", col, isIn, values)`` / ``("C", op, [children])``."""
    fi = getattr(compiled, "field_index", None) or {f: i for i, f in enumerate(compiled.active_fields)}
    schema = compiled.schema
    if isinstance(p, ir.TruePredicate):
        return ("T",)
    if isinstance(p, ir.FalsePredicate):
        return ("F",)
    if isinstance(p, ir.SimplePredicate):
        if p.operator in ("isMissing", "isNotMissing"):
            return ("M", fi[p.field], p.operator == "isMissing")
        if p.operator not in _OPS:
            raise NotLowerable(f"SimplePredicate operator {p.operator!r}")
        return ("S", fi[p.field], p.operator, float(schema.lookup(p.field, p.value)))
    if isinstance(p, ir.SimpleSetPredicate):
        return ("I", fi[p.field], p.boolean_operator == "isIn",
                [float(schema.lookup(p.field, v)) for v in p.values])
    return ("C", p.boolean_operator, [compile_predicate(q, compiled) for q in p.predicates])


_OPS = ("equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan", "greaterOrEqual")


def eval_predicate_device(prog, X):
    """``(true, unknown)`` boolean columns of a compiled predicate over the device matrix ``X``:
    fp64 comparisons of the fp32 inputs, the oracle's three-valued logic
    (`pmml/fields.py::eval_predicate`)."""
    import torch

    n = X.shape[0]
    ones = torch.ones(n, dtype=torch.bool, device=X.device)
    zeros = torch.zeros(n, dtype=torch.bool, device=X.device)
    tag = prog[0]
    if tag == "T":
        return ones, zeros
    if tag == "F":
        return zeros, zeros
    if tag == "M":
        miss = torch.isnan(X[:, prog[1]])
        return (miss if prog[2] else ~miss), zeros
    if tag == "S":
        x = X[:, prog[1]].double()
        miss = torch.isnan(x)
        v = prog[3]
        t = {"equal": x == v, "notEqual": x != v, "lessThan": x < v, "lessOrEqual": x <= v,
             "greaterThan": x > v, "greaterOrEqual": x >= v}[prog[2]]
        return t & ~miss, miss
    if tag == "I":
        x = X[:, prog[1]].double()
        miss = torch.isnan(x)
        inside = torch.isin(x, torch.tensor(prog[3], dtype=torch.float64, device=X.device))
        return (inside if prog[2] else ~inside) & ~miss, miss
    op = prog[1]
    parts = [eval_predicate_device(q, X) for q in prog[2]]
    if op == "surrogate":
        t, u = zeros.clone(), ones.clone()
        for pt, pu in parts:
            take = u & ~pu
            t = torch.where(take, pt, t)
            u = u & pu
        return t, u
    if op == "and":
        anyfalse, anyunk = zeros.clone(), zeros.clone()
        for pt, pu in parts:
            anyfalse |= ~pt & ~pu
            anyunk |= pu
        return ~anyfalse & ~anyunk, anyunk & ~anyfalse
    if op == "or":
        anytrue, anyunk = zeros.clone(), zeros.clone()
        for pt, pu in parts:
            anytrue |= pt
            anyunk |= pu
        return anytrue, anyunk & ~anytrue
    acc, unk = zeros.clone(), zeros.clone()  # xor
    for pt, pu in parts:
        acc ^= pt
        unk |= pu
    return acc & ~unk, unk


def probs_width(plan) -> Optional[int]:
    """Number of probability columns a classification plan writes through ``launch(probs=...)``
    (the oracle's ``ModelResult.probs`` of that model), or None when it cannot."""
    from .plans import EPI_ARGMAX, EPI_CUMULATIVE, EPI_LINKMAX, EPI_LOGISTIC2, EPI_SOFTMAX, LinearPlan, TreePlan

    inner = getattr(plan, "inner", None)
    if inner is not None:
        return probs_width(inner)
    if isinstance(plan, (LinearPlan, TreePlan)):
        e = getattr(plan, "epi_args", {})
        if e.get("mode") in (EPI_ARGMAX, EPI_SOFTMAX, EPI_CUMULATIVE, EPI_LOGISTIC2, EPI_LINKMAX):
            if isinstance(plan, TreePlan) and getattr(plan, "sharded", False):
                return None
            return 2 if e["mode"] == EPI_LOGISTIC2 else int(e.get("C", 0)) or None
        return None
    return None


def _index_outputs(plan) -> None:
    """Make a classification segment plan emit class *indices* (its epilogue's label table off)."""
    if getattr(plan, "table", None) is not None:
        plan.table = None
        plan.__dict__.pop("_args", None)
    inner = getattr(plan, "inner", None)
    if inner is not None:
        _index_outputs(inner)


_SP = dict(END=0, TRUE=1, FALSE=2, CMP=3, ISMISS=4, NOTMISS=5, SET=6, AND=7, OR=8, XOR=9, SURR=10)
_CMP = {"equal": 0, "notEqual": 1, "lessThan": 2, "lessOrEqual": 3, "greaterThan": 4, "greaterOrEqual": 5}
_METHOD_CODE = {"selectFirst": 0, "sum": 1, "average": 2, "weightedAverage": 3, "max": 4, "min": 5, "median": 6,
                "weightedMedian": 7, "majorityVote": 8, "weightedMajorityVote": 9}
_PROB_CODE = {"average": 10, "weightedAverage": 11, "max": 12, "median": 13}
SEG_MAXK = SEG_MAXC = 256  # ops/csrc/segment.hip: <64, 64> instantiation up to 64, <256, 256> beyond
SEG_STACK = 32  # seg_predicate's postfix stack: 2-bit entries of one uint64 (ops/csrc/segment.hip)
MULTI_MAX_TREES = 64  # tree segments this small share one pointer-layout launch (tree_pointer_multi_kernel)


def predicate_programs(progs) -> tuple:
    """The compiled segment predicates as the reduction kernel's postfix programs:
    ``(insns int32[m, 4], pool float64[p], starts int32[K])`` (``ops/csrc/segment.hip``)."""
    insns: List[tuple] = []
    pool: List[float] = []
    depth = [0, 0]  # running postfix stack depth, its maximum over the program

    def push(pops: int) -> None:
        depth[0] += 1 - pops
        depth[1] = max(depth[1], depth[0])

    def emit(prog) -> None:
        tag = prog[0]
        if tag != "C":
            push(0)
        if tag == "T":
            insns.append((_SP["TRUE"], 0, 0, 0))
        elif tag == "F":
            insns.append((_SP["FALSE"], 0, 0, 0))
        elif tag == "M":
            insns.append((_SP["ISMISS"] if prog[2] else _SP["NOTMISS"], prog[1], 0, 0))
        elif tag == "S":
            insns.append((_SP["CMP"] | (_CMP[prog[2]] << 8), prog[1], len(pool), 1))
            pool.append(float(prog[3]))
        elif tag == "I":
            insns.append((_SP["SET"] | ((1 if prog[2] else 0) << 8), prog[1], len(pool), len(prog[3])))
            pool.extend(float(v) for v in prog[3])
        else:
            if len(prog[2]) > 32:
                raise NotLowerable("CompoundPredicate with more than 32 children")
            if not prog[2]:
                raise NotLowerable("CompoundPredicate without children")
            for q in prog[2]:
                emit(q)
            push(len(prog[2]))
            insns.append(({"and": _SP["AND"], "or": _SP["OR"], "xor": _SP["XOR"], "surrogate": _SP["SURR"]}[prog[1]],
                          len(prog[2]), 0, 0))

    starts = []
    for prog in progs:
        starts.append(len(insns))
        depth[0] = depth[1] = 0
        emit(prog)
        # seg_predicate keeps its three-valued stack as 2-bit entries of one uint64: a program whose
        # postfix stack ever holds more than SEG_STACK entries would shift the oldest ones out
        if depth[1] > SEG_STACK:
            raise NotLowerable(f"segment predicate needs a {depth[1]}-entry stack > {SEG_STACK}")
        insns.append((_SP["END"], 0, 0, 0))
    return (np.array(insns, dtype=np.int32).reshape(-1, 4), np.array(pool or [0.0], dtype=np.float64),
            np.array(starts, dtype=np.int32))


class SegmentedPlan(DevicePlan):
    """Per-segment device plans + device predicates + tensor-op aggregation (module docstring)."""

    graph_small_batches = True  # several launches per call: HIP-graph replay for small batches (runtime/graphs.py)

    kind = "segmented"
    supports_direct = False
    _STATE = DevicePlan._STATE + ("method", "kind_", "skip", "weights", "progs", "remap_lists", "table", "tgt",
                                  "categories", "n_subs")

    def __init__(self, compiled, device, **opts):
        from .plans import compile_plan

        super().__init__(compiled, device)
        ev = compiled.evaluator
        why = segmentable(ev, compiled)
        if why:
            raise NotLowerable(why)
        if self.prep is not None:
            raise NotLowerable("segmented plans read prepared inputs (compile_plan adds the prepare pass)")
        self.method = ev.method
        self.kind_ = ev.kind
        self.skip = ev.mm.missing_prediction_treatment == "skipSegment"
        self.weights = [float(s.weight) for s in ev.segments]
        self.progs = [compile_predicate(s.predicate, compiled) for s in ev.segments]
        self.subs: List[DevicePlan] = []
        for seg, sub in zip(ev.segments, ev.sub):
            try:
                plan = compile_plan(SubView(compiled, sub), device, **dict(opts))
            except NotLowerable as e:
                raise NotLowerable(f"segment {seg.id!r}: {e}") from e
            if self.kind_ == "classification":
                if sub.kind != "classification":
                    raise NotLowerable("classification segmentation over non-classification segments")
                if self.method in PROB_METHODS and probs_width(plan) != len(sub.categories):
                    raise NotLowerable(f"segment {seg.id!r}: {type(plan).__name__} does not expose probabilities")
                _index_outputs(plan)
            self.subs.append(plan)
        self.n_subs = len(self.subs)
        self._pointer_segments(compiled, ev, device, opts)
        self.table, self.tgt, self.categories, self.remap_lists = None, None, None, None
        if self.kind_ == "classification":
            cats = list(ev.sub[0].categories) if self.method == "selectFirst" else list(ev.categories)
            self.remap_lists = [[cats.index(c) if c in cats else -1 for c in sub.categories] + [-1]
                                for sub in ev.sub]
            self.categories = cats
            self.table = self._t(_label_table(cats))
        elif ev.target is not None:
            self.tgt = target_post(ev.target, force=True)
        self._post_build()

    def _pointer_segments(self, compiled, ev, device, opts) -> None:
        """Small tree segments (<= MULTI_MAX_TREES trees in all) are re-lowered on the pointer
        layout, whose walk does not depend on the depth: they then score in ONE launch
        (``tree_pointer_multi_kernel``, grid.z = segment) instead of one launch each."""
        from .plans import TreePlan, compile_plan

        if "layout" in opts or self.n_subs < 2:
            return
        trees = [p for p in self.subs if isinstance(p, TreePlan)]
        if len(trees) < 2 or sum(p.n_trees for p in trees) > MULTI_MAX_TREES:
            return
        for i, (sub, plan) in enumerate(zip(ev.sub, self.subs)):
            if not isinstance(plan, TreePlan) or plan.layout == "pointer":
                continue
            try:
                new = compile_plan(SubView(compiled, sub), device, **dict(opts, layout="pointer"))
            except NotLowerable:
                continue
            if not isinstance(new, TreePlan) or new.layout != "pointer":
                continue
            if self.kind_ == "classification":
                if self.method in PROB_METHODS and probs_width(new) != probs_width(plan):
                    continue
                _index_outputs(new)
            self.subs[i] = new

    def _build_multi(self, probs: bool, coff) -> None:
        """Device argument blocks of the pointer-layout tree segments, one group per accumulator
        kind (single value / multi-slot), for pmml_tree_pointer_multi."""
        import torch

        from .plans import TreePlan

        self._multi = []
        # 16-byte BFS nodes only (the refill / compact / super / rank3 / LDS formats have kernels of
        # their own and inline-leaf nodes a different child encoding; the clamped, masked, uskip and
        # peel loads of the same nodes are bit-identical walks)
        own = (VAR_POINTER_REFILL | VAR_POINTER_COMPACT | VAR_POINTER_SUPER | VAR_POINTER_RANK3 | VAR_POINTER_LDS
               | VAR_POINTER_INLINE)
        members = [i for i, p in enumerate(self.subs)
                   if isinstance(p, TreePlan) and p.layout == "pointer" and p.C <= 16 and (int(p.variant) & own) == 0]
        if len(members) < 2:
            return
        for general in (0, 1):
            idx = [i for i in members if int(self.subs[i].general) == general]
            if not idx:
                continue
            blob = b"".join(bytes(self.subs[i]._args_template(probs)) for i in idx)
            segs = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.device)
            sidx = torch.tensor(idx, dtype=torch.int32, device=self.device)
            poff = torch.tensor([int(coff[i]) for i in idx], dtype=torch.int64, device=self.device) if probs else None
            self._multi.append(dict(general=general, idx=idx, segs=segs, sidx=sidx, poff=poff,
                                    max_c=max(int(self.subs[i].C) for i in idx)))

    def _post_build(self) -> None:
        import torch

        self.remaps = [torch.tensor(r, dtype=torch.int64, device=self.device) for r in (self.remap_lists or [])]
        self._multi = None  # built lazily by the first fused launch (the segments' args templates)
        # the fused reduction kernel's tables (ops/csrc/segment.hip); None -> tensor-op aggregation
        self._red = None
        probs = self.kind_ == "classification" and self.method in PROB_METHODS
        code = _PROB_CODE[self.method] if probs else _METHOD_CODE.get(self.method)
        if code is None or self.n_subs > SEG_MAXK or (self.categories and len(self.categories) > SEG_MAXC) or \
                any(len(r) - 1 > SEG_MAXC for r in (self.remap_lists or [])):
            return
        try:
            insns, pool, starts = predicate_programs(self.progs)
        except NotLowerable:
            return
        widest = max([self.n_subs, len(self.categories or [])] + [len(r) - 1 for r in (self.remap_lists or [])])
        stride = (64 if widest <= 64 else SEG_MAXC) + 1  # the kernel instantiation (remap row length)
        rm = np.full((max(1, self.n_subs), stride), -1, dtype=np.int32)
        for i, r in enumerate(self.remap_lists or []):
            rm[i, : len(r) - 1] = r[:-1]
        widths = [len(r) - 1 for r in self.remap_lists] if probs else [0] * self.n_subs
        coff = np.zeros(self.n_subs + 1, dtype=np.int64)
        np.cumsum(widths, out=coff[1:])
        dev = self.device
        self._red = dict(code=code, probs=probs, widths=widths, stride=stride,
                         prog=torch.from_numpy(insns.reshape(-1)).to(dev), pool=torch.from_numpy(pool).to(dev),
                         pc=torch.from_numpy(starts).to(dev),
                         weights=torch.tensor(self.weights, dtype=torch.float64, device=dev),
                         remap=torch.from_numpy(rm.reshape(-1)).to(dev), coff=torch.from_numpy(coff).to(dev),
                         coff_h=coff,
                         table=self.table if self.table is not None else torch.zeros(1, device=dev))

    # replication: the container's scalars + every segment plan's state under "sub<i>/"
    def export_state(self):
        meta, tensors = super().export_state()
        meta["sub_metas"] = []
        for i, plan in enumerate(self.subs):
            m, t = plan.export_state()
            meta["sub_metas"].append(m)
            for k, v in t.items():
                tensors[f"sub{i}/{k}"] = v
                meta["__tensors__"][f"sub{i}/{k}"] = (tuple(v.shape), str(v.dtype).replace("torch.", ""))
        return meta, tensors

    def _post_state(self) -> None:
        subs = []
        for i, m in enumerate(self.sub_metas):
            pre = f"sub{i}/"
            t = {k[len(pre):]: v for k, v in self.__dict__.items() if k.startswith(pre)}
            subs.append(DevicePlan.from_state(m, t, self.device))
        for k in [k for k in self.__dict__ if k.startswith("sub") and "/" in k]:
            del self.__dict__[k]
        self.subs = subs
        self._post_build()

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None, **kw) -> None:
        import torch

        if self.device.type == "cuda" and getattr(self, "_red", None) is not None:
            self._launch_fused(X, score, valid, stream, score2, valid2)
            return
        n = X.shape[0]
        if self.device.type == "cuda":
            st = stream if stream is not None else torch.cuda.current_stream(self.device)
            ctx = torch.cuda.stream(st)
        else:  # lowering dry run (CPU tests with stand-in segment plans)
            st, ctx = None, contextlib.nullcontext()
        with ctx:
            S = torch.empty((self.n_subs, n), dtype=torch.float32, device=self.device)
            V = torch.empty((self.n_subs, n), dtype=torch.uint8, device=self.device)
            probs = self.kind_ == "classification" and self.method in PROB_METHODS
            Pr = []
            for i, plan in enumerate(self.subs):
                if probs:
                    Pr.append(torch.full((n, len(self.remap_lists[i]) - 1), float("nan"), dtype=torch.float32,
                                         device=self.device))
                plan.launch(X, S[i], V[i], stream=st, **({"probs": Pr[i]} if probs else {}))
            T = torch.stack([eval_predicate_device(p, X)[0] for p in self.progs])  # [K, n] TRUE masks
            ok = V.bool() & ~torch.isnan(S)
            if self.method == "selectFirst":
                s, v = self._select(S, ok, T)
            elif probs:
                s, v = self._prob_combine(Pr, ok, T)
            elif self.kind_ == "classification":
                s, v = self._vote(S, ok, T)
            else:
                s, v = self._regress(S.double(), ok, T)
            s = torch.where(v, s, torch.full_like(s, float("nan")))
            for so, vo in ((score, valid), (score2, valid2)):
                if so is not None and not isinstance(so, int):
                    so.copy_(s.to(so.dtype))
                    vo.copy_(v.to(torch.uint8))

    def _launch_fused(self, X, score, valid, stream, score2, valid2) -> None:
        """Segment plans, then ONE kernel for predicates + aggregation + target / label epilogue."""
        import ctypes

        import torch

        from ..ops._lib import MultiTreeArgs, SegArgs, check, stream_handle
        from .plans import _addr

        n = X.shape[0]
        if n == 0:
            return
        r = self._red
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(st):
            S = torch.empty((self.n_subs, n), dtype=torch.float32, device=self.device)
            V = torch.empty((self.n_subs, n), dtype=torch.uint8, device=self.device)
            P = torch.empty(max(1, int(r["coff_h"][-1]) * n), dtype=torch.float32, device=self.device) \
                if r["probs"] else None
            done = set()
            if n and X.shape[1] <= 64 and X.stride(1) == 1 and X.dtype == torch.float32:
                if self._multi is None:
                    self._build_multi(r["probs"], r["coff_h"])
                for g in self._multi:
                    m = MultiTreeArgs()
                    m.segs, m.X, m.S, m.V = g["segs"].data_ptr(), X.data_ptr(), S.data_ptr(), V.data_ptr()
                    m.P = P.data_ptr() if P is not None else None
                    m.poff = g["poff"].data_ptr() if g["poff"] is not None else None
                    m.sidx = g["sidx"].data_ptr()
                    m.n_rows, m.n_feat, m.ldx, m.count = n, X.shape[1], X.stride(0), len(g["idx"])
                    check(self.lib.pmml_tree_pointer_multi(stream_handle(st), ctypes.byref(m), g["general"],
                                                           g["max_c"]), "multi-segment tree launch")
                    done.update(g["idx"])
            for i, plan in enumerate(self.subs):
                if i in done:
                    continue
                kw = {}
                if r["probs"]:
                    a0, w = int(r["coff_h"][i]) * n, r["widths"][i]
                    kw["probs"] = P[a0: a0 + n * w].view(n, w)
                plan.launch(X, S[i], V[i], stream=st, **kw)
            a = SegArgs()
            a.X, a.n_rows, a.ldx = X.data_ptr(), n, X.stride(0)
            a.S, a.V = S.data_ptr(), V.data_ptr()
            a.P = P.data_ptr() if P is not None else None
            a.coff, a.prog, a.pool, a.pc = (r["coff"].data_ptr(), r["prog"].data_ptr(), r["pool"].data_ptr(),
                                            r["pc"].data_ptr())
            a.weights, a.remap, a.table = r["weights"].data_ptr(), r["remap"].data_ptr(), r["table"].data_ptr()
            a.K, a.C = self.n_subs, len(self.categories or [])
            a.method, a.classification = r["code"], 1 if self.kind_ == "classification" else 0
            a.skip = 1 if self.skip else 0
            t = self.tgt
            a.tgt = int(t["flags"]) if t else 0
            if t:
                a.lo, a.hi, a.ta, a.tb, a.dflt = t["lo"], t["hi"], t["ta"], t["tb"], t["dflt"]
            else:
                a.ta = 1.0
            a.score, a.valid = _addr(score), _addr(valid)
            a.score2, a.valid2 = _addr(score2), _addr(valid2)
            a.remap_stride = int(r["stride"])
            check(self.lib.pmml_segment_reduce(stream_handle(st), ctypes.byref(a)), "segment reduce kernel")

    def _select(self, S, ok, T):
        import torch

        K, n = S.shape
        idx = torch.arange(K, device=S.device)[:, None].expand(K, n)
        first = torch.where(T, idx, torch.full_like(idx, K)).min(dim=0).values  # K: no segment
        hit = first < K
        f = first.clamp(max=K - 1)[None, :]
        s = S.gather(0, f)[0]
        v = ok.gather(0, f)[0] & hit
        if self.kind_ == "classification":
            seg_idx = torch.stack([r[torch.where(torch.isnan(S[i]), -1, S[i]).long().clamp(min=-1)]
                                   for i, r in enumerate(self.remaps)])
            lab = seg_idx.gather(0, f)[0]
            v = v & (lab >= 0)
            s = self.table[lab.clamp(min=0)].double()
            v = v & ~torch.isnan(s)
            return s, v
        s = s.double()
        s, v = apply_target_torch(s, v & torch.isfinite(s), self.tgt)
        return s, v

    def _regress(self, S, ok, T):
        import torch

        use = T & ok
        miss = T & ~ok
        m = self.method
        Vz = torch.where(use, S, torch.zeros_like(S))
        cnt = use.sum(dim=0)
        if m == "sum":
            out = Vz.sum(dim=0)
        elif m == "average":
            out = Vz.sum(dim=0) / cnt
        elif m == "weightedAverage":
            w = torch.tensor(self.weights, dtype=torch.float64, device=S.device)[:, None]
            out = (Vz * w).sum(dim=0) / torch.where(use, w.expand_as(S), torch.zeros_like(S)).sum(dim=0)
        elif m in ("max", "min"):
            fill = float("-inf") if m == "max" else float("inf")
            Vf = torch.where(use, S, torch.full_like(S, fill))
            out = Vf.max(dim=0).values if m == "max" else Vf.min(dim=0).values
        elif m == "weightedMedian":  # first value whose cumulative weight reaches half the total
            w = torch.tensor(self.weights, dtype=torch.float64, device=S.device)[:, None].expand_as(S)
            srt, order = torch.where(use, S, torch.full_like(S, float("inf"))).sort(dim=0, stable=True)
            cw = torch.where(use, w, torch.zeros_like(w)).gather(0, order).cumsum(dim=0)
            below = (cw < 0.5 * cw[-1:]).sum(dim=0).clamp(max=S.shape[0] - 1)
            out = srt.gather(0, below[None, :])[0]
        else:  # median: mean of the two middle values of the participating segments (numpy rule)
            out = _median0(torch.where(use, S, torch.full_like(S, float("nan"))))
        v = cnt > 0
        if not self.skip:
            v = v & ~miss.any(dim=0)
        v = v & torch.isfinite(out)
        out, v = apply_target_torch(out, v, self.tgt)
        return out, v

    def _prob_combine(self, Pr, ok, T):
        """Classification ``average`` / ``weightedAverage`` / ``max`` / ``median`` over segment
        probabilities (oracle: ``MiningEvaluator._classify``)."""
        import torch

        K, n = ok.shape
        C = len(self.categories)
        use = T & ok
        anymiss = (T & ~ok).any(dim=0)
        m = self.method
        fill = float("nan") if m == "median" else 0.0
        P = torch.full((K, n, C), fill, dtype=torch.float64, device=ok.device)
        for i in range(K):
            cols = self.remaps[i][:-1]
            keep = cols >= 0
            src = Pr[i].double()
            if m != "median":
                src = torch.nan_to_num(src, nan=0.0)
            P[i][:, cols[keep]] = src[:, keep]
        if m in ("average", "weightedAverage"):
            w = torch.tensor([w if m == "weightedAverage" else 1.0 for w in self.weights], dtype=torch.float64,
                             device=ok.device)[:, None]
            wu = torch.where(use, w.expand(K, n), torch.zeros((K, n), dtype=torch.float64, device=ok.device))
            probs = (P * wu[:, :, None]).sum(dim=0) / wu.sum(dim=0)[:, None]
        elif m == "max":
            probs = torch.where(use[:, :, None], P, torch.zeros_like(P)).max(dim=0).values.clamp(min=0.0)
        else:
            probs = _median0(torch.where(use[:, :, None], P, torch.full_like(P, float("nan"))))
        v = use.any(dim=0)
        if not self.skip:
            v = v & ~anymiss
        lab = torch.nan_to_num(probs, nan=-1.0).argmax(dim=1)  # ties -> lowest index, as np.argmax
        s = self.table[lab].double()
        return s, v & ~torch.isnan(s)

    def _vote(self, S, ok, T):
        import torch

        K, n = S.shape
        C = len(self.categories)
        use = T & ok
        anymiss = (T & ~ok).any(dim=0)
        acc = torch.zeros((n, C), dtype=torch.float64, device=S.device)
        for i in range(K):
            lab = self.remaps[i][torch.where(use[i], S[i], torch.zeros_like(S[i])).long()]
            w = self.weights[i] if self.method == "weightedMajorityVote" else 1.0
            u = use[i] & (lab >= 0)
            acc.scatter_add_(1, lab.clamp(min=0)[:, None], torch.where(u, w, 0.0).double()[:, None])
        v = use.any(dim=0)
        if not self.skip:
            v = v & ~anymiss
        lab = acc.argmax(dim=1)  # ties -> lowest index, as np.argmax
        s = self.table[lab].double()
        return s, v & ~torch.isnan(s)


class ChainView(SubView):
    """A chain segment's model over its own MiningSchema's active fields, which may include the
    Output fields of earlier segments (columns of the chain's augmented matrix)."""

    def __init__(self, parent, evaluator, columns: List[str]):
        super().__init__(parent, evaluator)
        self.active_fields = list(columns)
        self.field_index = {c: j for j, c in enumerate(columns)}

    @property
    def n_features(self) -> int:
        return len(self.active_fields)


_CHAIN_OUT = ("predictedValue", "transformedValue", "probability", "decision")


class ChainPlan(DevicePlan):
    """``multipleModelMethod="modelChain"`` beyond the fused tree → calibrator form: the segments
    run in document order on an augmented device matrix ``[inputs | chain outputs]``; each
    segment's Output fields are written into their columns where its predicate is TRUE (NaN
    elsewhere, as the oracle hides them), later segments read them like inputs, and every row takes
    the result of the LAST segment whose predicate is TRUE (`models/mining.py::MiningEvaluator._select`).

    Output fields: predictedValue (classification segments score class INDICES here; a per-output
    table maps them to the field's encoding, so string-typed labels feed later segments as their
    vocabulary codes, as in the oracle), probability of a class, transformedValue / decision
    without an expression (the segment value), and transformedValue / decision WITH an expression:
    those are compiled into one derive program per segment (``ops/csrc/derive.hip``, the postfix
    fp64 VM of the DerivedField pass) over the augmented columns — they may read inputs, earlier
    segments' outputs and this segment's own outputs, in document order like
    ``ModelEvaluator.compute_outputs``."""

    kind = "chain"
    supports_direct = False

    def __init__(self, compiled, device, **opts):
        from .plans import compile_plan

        super().__init__(compiled, device)
        ev = compiled.evaluator
        if not isinstance(ev, MiningEvaluator) or ev.method != "modelChain":
            raise NotLowerable("not a modelChain")
        if self.prep is not None:
            raise NotLowerable("chain plans read prepared inputs (compile_plan adds the prepare pass)")
        schema = compiled.schema
        base = list(compiled.active_fields)
        self.n_base = len(base)
        # (segment, column, feature, class position or -1, value table index or -1, expression or None)
        self.outs = []
        self.tables: List[np.ndarray] = []
        names = list(base)
        for i, (seg, sub) in enumerate(zip(ev.segments, ev.sub)):
            cats = list(getattr(sub, "categories", None) or []) if sub.kind == "classification" else []
            for of in sub.model.output:
                if of.feature not in _CHAIN_OUT:
                    raise NotLowerable(f"chain output {of.name!r}: feature {of.feature!r} is host-only")
                if of.name in names:
                    raise NotLowerable(f"chain output {of.name!r} shadows a field")
                pos, tab, ex = -1, -1, None
                if of.feature == "probability":
                    if of.value is None or of.value not in cats:
                        raise NotLowerable(f"chain output {of.name!r}: probability of an unknown class")
                    pos = cats.index(of.value)
                elif of.feature in ("transformedValue", "decision") and of.expression is not None:
                    ex = of.expression
                elif of.feature == "decision":
                    raise NotLowerable(f"chain output {of.name!r}: decision without an expression")
                elif of.feature == "transformedValue":
                    pos = -2 if sub.kind == "classification" else -1  # -2: the oracle's NaN column
                elif sub.kind == "classification":
                    # class index -> the output field's encoding of the label (a vocabulary code for a
                    # string-typed field, the label's number otherwise)
                    tab = len(self.tables)
                    self.tables.append(np.array([schema.lookup(of.name, c) for c in cats] + [np.nan]))
                elif sub.kind == "regression":
                    pass
                else:
                    raise NotLowerable(f"chain output {of.name!r}: {sub.kind} predictedValue is host-only")
                self.outs.append((i, len(names), of.feature, pos, tab, ex))
                names.append(of.name)
        self.columns = names
        col = {c: j for j, c in enumerate(names)}
        self.progs = [compile_predicate(s.predicate, _Cols(compiled, col)) for s in ev.segments]
        self.subs, self.cols, self.need_probs, self.label_tabs = [], [], [], []
        for i, (seg, sub) in enumerate(zip(ev.segments, ev.sub)):
            used = [f.name for f in sub.model.mining_schema.active]
            missing = [f for f in used if f not in col]
            if missing:
                raise NotLowerable(f"chain segment {seg.id!r} reads unknown fields {missing}")
            try:
                plan = compile_plan(ChainView(compiled, sub, used), device, **dict(opts))
            except NotLowerable as e:
                raise NotLowerable(f"chain segment {seg.id!r}: {e}") from e
            want = any(o[0] == i and o[2] == "probability" for o in self.outs)
            if want and probs_width(plan) != len(sub.categories):
                raise NotLowerable(f"chain segment {seg.id!r}: {type(plan).__name__} does not expose probabilities")
            if sub.kind == "classification":
                _index_outputs(plan)  # class indices; labels through label_tabs / output tables
                self.label_tabs.append(self._t(np.append(_label_table(list(sub.categories)), np.float32(np.nan))))
            else:
                self.label_tabs.append(None)
            self.subs.append(plan)
            self.cols.append([col[f] for f in used])
            self.need_probs.append(len(sub.categories) if want else 0)
        # expression outputs: one derive program per segment over every augmented column
        self.expr_progs = [self._expr_program(compiled, col, i) for i in range(len(self.subs))]
        self.kind_ = ev.kind
        final = ev.sub[-1]
        self.tgt = target_post(ev.target, force=True) if ev.kind == "regression" and ev.target is not None else None
        self.final_labels = None
        if ev.kind == "classification":
            self.final_labels = self._t(_label_table(list(final.categories)))
        self._col_idx = [self._t(np.array(c, dtype=np.int64)) for c in self.cols]
        self._tabs = [self._t(t) for t in self.tables]

    def _expr_program(self, compiled, col: dict, seg: int):
        """``(DerivedProgram, insns, pool, out_cols, [augmented column of each output])`` computing
        segment ``seg``'s expression outputs in document order, or None."""
        from .derive import INSN_DTYPE, OP_STORE, STACK_DEPTH, DerivedProgram, _Emitter

        exprs = [(c, ex) for s_, c, _, _, _, ex in self.outs if s_ == seg and ex is not None]
        if not exprs:
            return None
        n_in = len(self.columns)
        if n_in + len(exprs) > 256:
            raise NotLowerable("chain expression outputs: more than 256 augmented columns")
        col_of = dict(col)
        em = _Emitter(compiled.schema, col_of)
        derived = []
        for j, (c, ex) in enumerate(exprs):
            name = self.columns[c]
            em.expr(ex, name)
            dt = compiled.schema.types.get(name)
            em.emit(OP_STORE, a=n_in + j, c=2 if dt == "integer" else 0, pops=1)
            col_of[name] = n_in + j  # later expressions read the fresh value
            derived.append(name)
        if em.max_sp > STACK_DEPTH:
            raise NotLowerable(f"chain expression output needs a stack of {em.max_sp} > {STACK_DEPTH}")
        insns = np.array(em.insns, dtype=INSN_DTYPE)
        prog = DerivedProgram(list(self.columns), derived, derived, insns, np.array(em.pool or [0.0]), em.max_sp)
        return (prog, self._t(insns.view(np.int32).reshape(-1)), self._t(prog.pool), self._t(prog.out_cols),
                [c for c, _ in exprs])

    def _run_expr(self, ep, Xa, st):
        """The derive program over the augmented matrix -> ``[n, outputs]`` fp32."""
        import ctypes

        import torch

        from ..ops._lib import DeriveArgs, check, ptr, stream_handle
        from .derive import emulate

        prog, insns, pool, out_cols, _ = ep
        n = Xa.shape[0]
        if self.device.type != "cuda":  # lowering dry run (CPU tests): the kernel's numpy twin
            return torch.from_numpy(emulate(prog, Xa.double().numpy()))
        out = torch.empty((n, len(prog.selected)), dtype=torch.float32, device=self.device)
        ok = torch.empty(n, dtype=torch.uint8, device=self.device)
        a = DeriveArgs()
        a.X = Xa.data_ptr()
        a.n_rows, a.n_in, a.ldx, a.n_tile = n, Xa.shape[1], Xa.stride(0), prog.n_tile
        a.prep, a.prog, a.pool, a.out_cols = None, ptr(insns), ptr(pool), ptr(out_cols)
        a.n_insn, a.n_sel = len(prog.insns), len(prog.selected)
        a.out, a.row_ok = ptr(out), ptr(ok)
        check(self.lib.pmml_derive_launch(stream_handle(st), ctypes.byref(a)), "chain output derive kernel")
        return out

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None, **kw) -> None:
        import torch

        n = X.shape[0]
        if n == 0:
            return
        st = stream if stream is not None and self.device.type == "cuda" else None
        ctx = torch.cuda.stream(st) if st is not None else contextlib.nullcontext()
        nan = float("nan")
        with ctx:
            Xa = torch.full((n, len(self.columns)), nan, dtype=torch.float32, device=self.device)
            Xa[:, : self.n_base] = X[:, : self.n_base]
            best_s = torch.full((n,), nan, dtype=torch.float64, device=self.device)
            best_v = torch.zeros(n, dtype=torch.bool, device=self.device)
            for i, plan in enumerate(self.subs):
                Xi = Xa.index_select(1, self._col_idx[i]).contiguous()
                if Xi.shape[1] == 0:  # a segment without inputs: never hand a kernel a 0-wide matrix
                    Xi = torch.zeros((n, 1), dtype=torch.float32, device=self.device)
                s = torch.empty(n, dtype=torch.float32, device=self.device)
                v = torch.empty(n, dtype=torch.uint8, device=self.device)
                pr = None
                if self.need_probs[i]:
                    pr = torch.full((n, self.need_probs[i]), nan, dtype=torch.float32, device=self.device)
                plan.launch(Xi, s, v, stream=st, **({"probs": pr} if pr is not None else {}))
                t = eval_predicate_device(self.progs[i], Xa)[0]
                ok = v.bool() & ~torch.isnan(s)  # the segment predicted (its outputs exist)
                idx = None
                lab_ok = ok
                if self.label_tabs[i] is not None:  # class index -> label (NaN: not a number)
                    k = self.label_tabs[i].numel() - 1
                    idx = torch.where(ok, s, torch.full_like(s, float(k))).long().clamp(0, k)
                    s = self.label_tabs[i][idx]
                    lab_ok = ok & ~torch.isnan(s)
                mine = []
                for seg, c, feat, pos, tab, ex in self.outs:  # the values, unmasked by the predicate
                    if seg != i or ex is not None:
                        continue
                    if feat == "probability":
                        val = pr[:, pos]
                    elif tab >= 0:
                        val = self._tabs[tab][idx].float()
                    elif pos == -2:
                        val = torch.full_like(s, nan)
                    else:
                        val = s
                    Xa[:, c] = torch.where(ok, val, torch.full_like(val, nan))
                    mine.append(c)
                ep = self.expr_progs[i]
                if ep is not None:  # expression outputs see this segment's own outputs (document order)
                    out = self._run_expr(ep, Xa, st)
                    for j, c in enumerate(ep[4]):
                        Xa[:, c] = out[:, j].to(Xa.dtype)
                        mine.append(c)
                if mine:  # rows the segment does not apply to do not see its outputs
                    cols = torch.tensor(mine, dtype=torch.int64, device=self.device)
                    Xa[:, cols] = torch.where(t[:, None], Xa[:, cols], torch.full_like(Xa[:, cols], nan))
                best_s = torch.where(t, s.double(), best_s)  # the last applicable segment wins
                best_v = torch.where(t, lab_ok, best_v)
            if self.kind_ == "classification":
                best_v = best_v & torch.isin(best_s.float(), self.final_labels)
            else:
                best_v = best_v & torch.isfinite(best_s)
                best_s, best_v = apply_target_torch(best_s, best_v, self.tgt)
            out = torch.where(best_v, best_s, torch.full_like(best_s, nan))
            for so, vo in ((score, valid), (score2, valid2)):
                if so is not None and not isinstance(so, int):
                    so.copy_(out.to(so.dtype))
                    vo.copy_(best_v.to(torch.uint8))


class _Cols:
    """compile_predicate's view of the chain's augmented columns."""

    def __init__(self, compiled, index):
        self.field_index = index
        self.active_fields = list(index)
        self.schema = compiled.schema


def _median0(A):
    """``numpy.nanmedian`` along dim 0 (mean of the two middle values; NaN where nothing is left)."""
    import torch

    cnt = (~torch.isnan(A)).sum(dim=0)
    srt = torch.where(torch.isnan(A), torch.full_like(A, float("inf")), A).sort(dim=0).values
    c = cnt.clamp(min=1)
    lo = srt.gather(0, ((c - 1) // 2).unsqueeze(0))[0]
    hi = srt.gather(0, (c // 2).unsqueeze(0))[0]
    return torch.where(cnt > 0, (lo + hi) / 2, torch.full_like(lo, float("nan")))


__all__ = ["ChainPlan", "ChainView", "SegmentedPlan", "SubView", "probs_width", "segmentable"]
