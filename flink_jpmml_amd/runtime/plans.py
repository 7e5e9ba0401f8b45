"""Device plans: lowering of a :class:`CompiledPmml` into HIP-kernel operands on one GPU.

A plan owns device-resident model tensors (tree blobs, centres, weights, field-preparation
table) and exposes

* :meth:`DevicePlan.launch` — enqueue scoring of a device ``[rows, F]`` fp32 matrix on a HIP
  stream, writing ``score`` (fp32) and ``valid`` (u8) — no host synchronisation, graph-capturable;
* :meth:`DevicePlan.score` — convenience host/device entry point.

Numerics: inputs are fp32 on the device. Every fp64 constant that is compared against an input
(split thresholds, validity intervals) is rounded *directionally* to fp32 so the fp32 comparison
gives exactly the fp64 answer for any fp32 input (``_ceil32``/``_floor32``/``_next_up``).
Accumulations (tree sums, dot products) run in fp32; the parity tolerance against the float64
oracle is documented per test.
"""

from __future__ import annotations

import dataclasses
import logging
import math
import threading
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..models.clustering import ClusteringEvaluator
from ..models.mining import MiningEvaluator
from ..models.regression import RegressionEvaluator
from ..models.tree import OP_GE, OP_GT, OP_LE, OP_LT, BinaryTree, NotBinary, TreeEvaluator, lower_binary_tree
from ..pmml import ir

logger = logging.getLogger(__name__)

TB = 256  # rows per workgroup of every row-tile kernel (mirrors csrc)

# FieldPrep flag bits (mirror of csrc/common.h)
FP_HAS_MISSING_REPL = 1 << 0
FP_HAS_INTERVAL = 1 << 1
FP_LO_OPEN = 1 << 2
FP_HI_OPEN = 1 << 3
FP_INVALID_RETURN = 1 << 4
FP_INVALID_AS_MISSING = 1 << 5
FP_INVALID_AS_VALUE = 1 << 6
FP_OUTLIER_AS_MISSING = 1 << 7
FP_OUTLIER_AS_EXTREME = 1 << 8
FP_INTEGER = 1 << 9
FP_CODE_RANGE = 1 << 10
FP_ROW_INVALID = 1 << 11
FP_MISSING_VALUE = 1 << 12
FP_VALUE_MASK = 1 << 13
FP_VALUE_LIST = 1 << 14
MAX_VALUE_LIST = 255  # per list (8-bit counts in the FieldPrep pad word)

EPI_AFFINE, EPI_LOGISTIC2, EPI_ARGMAX, EPI_SOFTMAX, EPI_CUMULATIVE, EPI_LINKMAX = 0, 1, 2, 3, 4, 5
LINKS = {"none": 0, None: 0, "logit": 1, "exp": 2, "probit": 3, "cloglog": 4, "loglog": 5, "cauchit": 6}


class NotLowerable(UnsupportedFeatureException):
    """The model (or one of its fields) uses a feature the device path does not implement."""


# --------------------------------------------------------------------------- fp32 rounding


def _f32(x: float) -> np.float32:
    return np.float32(x)


def _ceil32(t: float) -> float:
    f = np.float32(t)
    if np.isfinite(t) and float(f) < t:
        f = np.nextafter(f, np.float32(np.inf))
    return float(f)


def _floor32(t: float) -> float:
    f = np.float32(t)
    if np.isfinite(t) and float(f) > t:
        f = np.nextafter(f, np.float32(-np.inf))
    return float(f)


def _next_up32(f: float) -> float:
    return float(np.nextafter(np.float32(f), np.float32(np.inf)))


def canonical_threshold(op: int, t: float) -> Tuple[float, bool]:
    """Return ``(T, swap)`` such that for every fp32 x: the original "go to first child" test
    equals ``not (x >= T)`` when ``swap`` is False, or ``x >= T`` when ``swap`` is True."""
    if op == OP_LT:  # left iff x < t  <=> right iff x >= t
        return _ceil32(t), False
    if op == OP_LE:  # left iff x <= t <=> right iff x > t <=> x >= nextup(floor32(t))
        return _next_up32(_floor32(t)), False
    if op == OP_GT:  # first iff x > t  -> first child goes RIGHT
        return _next_up32(_floor32(t)), True
    if op == OP_GE:  # first iff x >= t
        return _ceil32(t), True
    raise ValueError(op)


# --------------------------------------------------------------------------- field preparation


def _fp32_values(name: str, texts, what: str) -> List[float]:
    """The numeric members of a DataField Value list as fp32-exact numbers (non-numeric entries
    never reach a numeric matrix: the text parsers read them as missing, as ``prepare_matrix``
    skips them); a member fp32 cannot hold exactly is host-only."""
    out = []
    for txt in texts:
        try:
            v = float(txt)
        except ValueError:
            continue
        if not math.isfinite(v) or float(np.float32(v)) != v:
            raise NotLowerable(f"field {name!r}: {what} value {v!r} is not an fp32 number")
        out.append(v)
    if len(out) > MAX_VALUE_LIST:
        raise NotLowerable(f"field {name!r}: more than {MAX_VALUE_LIST} {what} values")
    return sorted(set(out), key=out.index)


def build_field_prep(compiled, fields: List[str]) -> Tuple[np.ndarray, bool]:
    """FieldPrep table for the active fields: ``[F, 8]`` raw 32-bit words (one 32-byte record per
    field), followed by the fp32 value lists of ``FP_VALUE_LIST`` fields (several missing-value
    sentinels, invalid-value lists) in extra 8-word rows of the same buffer — a record finds its
    lists through the relative offset in its pad word. Second value: whether any field needs
    preparation at all."""
    schema = compiled.schema
    table = np.zeros((len(fields), 8), dtype=np.float32)
    flags = np.zeros(len(fields), dtype=np.uint32)
    any_prep = False
    masks = {}  # field -> (bits 0-31, bits 32-63) of an FP_VALUE_MASK set, written as raw words
    lists = {}  # field -> (missing values, invalid values) of an FP_VALUE_LIST field
    for j, name in enumerate(fields):
        df = schema.data_fields.get(name)
        mf = compiled.mining_fields.get(name)
        fl = 0
        lo, hi = -np.inf, np.inf
        out_lo, out_hi = -np.inf, np.inf
        mrepl = math.nan
        irepl = math.nan
        mval = 0.0
        optype = (mf.optype if mf is not None and mf.optype else None) or (df.optype if df else "continuous")
        constrained = False
        if df is not None:
            if optype != "continuous" and df.intervals:
                fl |= FP_ROW_INVALID
            # numeric missing-value sentinels (e.g. -999) and invalid-value lists, compared in fp32
            # (prepare_matrix's order: a missing value first, then an invalid one). A string field's
            # lists are text: its matrix column holds vocabulary codes, and the text ingest already
            # read a listed missing token as missing -- prepare_matrix ignores them, and so does this
            sentinels = [] if df.is_string else _fp32_values(name, df.missing_values, "missing")
            invalids = [] if df.is_string else _fp32_values(name, df.invalid_values, "invalid")
            if len(sentinels) == 1 and not invalids:
                fl |= FP_MISSING_VALUE
                mval = sentinels[0]
            elif sentinels or invalids:
                fl |= FP_VALUE_LIST
                lists[j] = (sentinels, invalids)
                if invalids:
                    constrained = True
            if optype == "continuous" and df.intervals:
                if len(df.intervals) != 1:
                    raise NotLowerable(f"field {name!r}: multiple validity intervals are host-only")
                iv = df.intervals[0]
                fl |= FP_HAS_INTERVAL
                constrained = True
                lo_open = not iv.closure.startswith("closed")
                hi_open = not iv.closure.endswith("Closed")
                if df.data_type == "float":
                    # fp32 inputs: directional rounding makes the fp32 test exact
                    if iv.left is not None:
                        lo = _floor32(iv.left) if lo_open else _ceil32(iv.left)
                    if iv.right is not None:
                        hi = _ceil32(iv.right) if hi_open else _floor32(iv.right)
                else:
                    # fp64 inputs arrive rounded-to-nearest: rounding the bounds the same way keeps
                    # every valid value valid (monotonic rounding); only values within half an
                    # fp32 ulp outside a bound can be misclassified
                    if iv.left is not None:
                        lo = float(np.float32(iv.left))
                    if iv.right is not None:
                        hi = float(np.float32(iv.right))
                fl |= (FP_LO_OPEN if lo_open else 0) | (FP_HI_OPEN if hi_open else 0)
            elif df.values and df.is_string:
                fl |= FP_CODE_RANGE
                hi = float(len(df.values))
                constrained = True
            elif df.values and optype != "continuous":
                # label-encoded numeric categories: a contiguous run of integers is "integral and
                # inside [min, max]" (the oracle's set test); other sets stay host-only
                try:
                    vals = sorted({float(v) for v in df.values})
                except ValueError:
                    raise NotLowerable(f"field {name!r}: non-numeric valid value on a numeric field") from None
                if not all(v == math.floor(v) and abs(v) < 2 ** 24 for v in vals):
                    raise NotLowerable(f"field {name!r}: non-integral numeric valid values are host-only")
                if vals[-1] - vals[0] == len(vals) - 1:
                    fl |= FP_HAS_INTERVAL | FP_INTEGER
                    lo, hi = vals[0], vals[-1]
                elif vals[-1] - vals[0] < 64:  # a sparse set within 64 consecutive integers: bit mask
                    fl |= FP_VALUE_MASK
                    lo = vals[0]
                    bits = sum(1 << int(v - lo) for v in vals)
                    masks[j] = (bits & 0xFFFFFFFF, bits >> 32)
                else:
                    raise NotLowerable(f"field {name!r}: numeric valid values span more than 64 integers")
                constrained = True
            elif df.values:
                raise NotLowerable(f"field {name!r}: numeric valid-value lists on a continuous field are host-only")
            if df.data_type == "integer":
                fl |= FP_INTEGER
                constrained = True
        if mf is not None:
            if constrained:
                t = mf.invalid_value_treatment
                if t == "returnInvalid":
                    fl |= FP_INVALID_RETURN
                elif t == "asMissing":
                    fl |= FP_INVALID_AS_MISSING
                elif t == "asValue" and mf.invalid_value_replacement is not None:
                    fl |= FP_INVALID_AS_VALUE
                    irepl = schema.lookup(name, mf.invalid_value_replacement)
            if optype == "continuous" and mf.outliers in ("asMissingValues", "asExtremeValues"):
                fl |= FP_OUTLIER_AS_MISSING if mf.outliers == "asMissingValues" else FP_OUTLIER_AS_EXTREME
                if mf.low_value is not None:
                    out_lo = mf.low_value
                if mf.high_value is not None:
                    out_hi = mf.high_value
            if mf.missing_value_replacement is not None:
                fl |= FP_HAS_MISSING_REPL
                mrepl = schema.lookup(name, mf.missing_value_replacement)
        elif constrained:
            fl |= FP_INVALID_RETURN
        flags[j] = fl
        table[j, 1:8] = [lo, hi, mrepl, irepl, out_lo, out_hi, mval]
        any_prep = any_prep or fl != 0
    raw = table.view(np.uint32).copy()
    raw[:, 0] = flags
    for j, (w0, w1) in masks.items():
        raw[j, 5], raw[j, 6] = w0, w1
    if lists:
        pool: List[float] = []
        for j, (miss_v, inv_v) in lists.items():
            start = len(fields) * 8 + len(pool)  # in words from the start of the buffer
            off = start - j * 8  # relative to field j's record
            if off >= 1 << 16:
                raise NotLowerable("FieldPrep value lists too large")
            raw[j, 7] = off | (len(miss_v) << 16) | (len(inv_v) << 24)
            pool.extend(miss_v)
            pool.extend(inv_v)
        pad = np.zeros(-(-len(pool) // 8) * 8, dtype=np.float32)
        pad[: len(pool)] = pool
        raw = np.concatenate([raw, pad.view(np.uint32).reshape(-1, 8)], axis=0)
    return raw, any_prep


# --------------------------------------------------------------------------- plan base


_DRY_RUN = 0


class lowering_dry_run:
    """Context manager: build plans on ``device="cpu"`` without the HIP library, so CPU tests can
    inspect a plan's lowering decisions and emulate its kernel on the packed tensors."""

    def __enter__(self):
        global _DRY_RUN
        _DRY_RUN += 1
        return self

    def __exit__(self, *exc):
        global _DRY_RUN
        _DRY_RUN -= 1
        return False


class DevicePlan:
    kind = "base"
    supports_direct = False  # kernel can write zero-copy host outputs + device mirror

    def __init__(self, compiled, device):
        import torch

        from ..ops import _lib

        self.compiled = compiled
        self.device = torch.device(device)
        if self.device.type == "cpu" and _DRY_RUN:
            self.lib = None  # lowering only: tensors stay on the host, launch() is unavailable
        elif self.device.type != "cuda":
            raise ValueError(f"device plans need a cuda (HIP) device, got {self.device}")
        else:
            self.lib = _lib.load()
        self.n_features = compiled.n_features
        if getattr(compiled, "prepared_inputs", False):
            self.prep = None  # a derive pass already applied the MiningField preparation
        else:
            prep, any_prep = build_field_prep(compiled, compiled.active_fields)
            self.prep = torch.from_numpy(prep.view(np.int32)).to(self.device) if any_prep else None

    # -- helpers
    def _t(self, arr, dtype=None):
        import torch

        t = torch.as_tensor(np.ascontiguousarray(arr))
        if dtype is not None:
            t = t.to(dtype)
        return t.to(self.device)

    _STATE: Tuple[str, ...] = ("n_features", "prep")

    def launch(self, X, score, valid, stream=None, probs=None) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    # -- replication (rank 0 lowers, other ranks receive the tensors over RCCL)
    def export_state(self) -> Tuple[dict, dict]:
        import torch

        meta, tensors = {"__class__": type(self).__name__}, {}
        for k in self._STATE:
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                tensors[k] = v
            else:
                meta[k] = v
        meta["__tensors__"] = {k: (tuple(t.shape), str(t.dtype).replace("torch.", "")) for k, t in tensors.items()}
        meta["__none__"] = [k for k in self._STATE if getattr(self, k) is None]
        return meta, tensors

    @staticmethod
    def from_state(meta: dict, tensors: dict, device) -> "DevicePlan":
        import torch

        from ..ops import _lib

        cls = {c.__name__: c for c in (TreePlan, ClusterPlan, KnnPlan, LinearPlan)}.get(meta["__class__"])
        if cls is None and meta["__class__"] == "DerivedPlan":
            from .derive import DerivedPlan as cls
        if cls is None and meta["__class__"] == "SegmentedPlan":
            from .segmented import SegmentedPlan as cls
        if cls is None and meta["__class__"] == "SvmGemmPlan":
            from .nn_plans import SvmGemmPlan as cls
        if cls is None:
            from . import nn_plans

            cls = getattr(nn_plans, meta["__class__"])
        obj = cls.__new__(cls)
        obj.compiled = None
        obj.device = torch.device(device)
        obj.lib = _lib.load()
        for k, v in meta.items():
            if not k.startswith("__"):
                setattr(obj, k, v)
        for k in meta.get("__none__", []):
            setattr(obj, k, None)
        for k, t in tensors.items():
            setattr(obj, k, t.to(obj.device))
        obj._post_state()
        return obj

    def _post_state(self) -> None:
        pass

    def alloc_outputs(self, n: int):
        import torch

        return (torch.empty(n, dtype=torch.float32, device=self.device),
                torch.empty(n, dtype=torch.uint8, device=self.device))

    def score(self, X: Any, replace_nan: Optional[float] = None, stream=None, absent: Any = None):
        """Score a host (numpy) or device (torch) matrix; returns device tensors ``(score, valid)``.
        ``replace_nan`` fills the ``absent`` entries (every NaN when no mask is given)."""
        import torch

        if isinstance(X, np.ndarray):
            Xt = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(self.device, non_blocking=False)
        else:
            Xt = X.to(self.device, dtype=torch.float32)
        if Xt.dim() != 2 or Xt.shape[1] != self.n_features:
            raise ValueError(f"expected [rows, {self.n_features}] input, got {tuple(Xt.shape)}")
        Xt = Xt.contiguous()
        if replace_nan is not None:
            if absent is None:
                Xt = torch.nan_to_num(Xt, nan=float(replace_nan))
            else:
                mask = torch.as_tensor(np.asarray(absent, dtype=bool)).to(self.device)
                Xt = torch.where(mask, torch.full_like(Xt, float(replace_nan)), Xt)
        score, valid = self.alloc_outputs(Xt.shape[0])
        self.launch(Xt, score, valid, stream=stream)
        return score, valid.bool()


def _epilogue(mode: int, C: int = 1, a: float = 1.0, b: float = 0.0, thr: float = 0.5, table=None,
              write_probs: bool = False, link: int = 0, tgt: Optional[dict] = None):
    from ..ops._lib import Epilogue

    e = Epilogue()
    e.mode, e.n_classes, e.a, e.b, e.thr = mode, C, a, b, thr
    e.has_table = 1 if table is not None else 0
    e.table = table.data_ptr() if table is not None else None
    e.write_probs = 1 if write_probs else 0
    e.link = link
    if tgt:
        e.tgt, e.lo, e.hi, e.ta, e.tb, e.dflt = tgt["flags"], tgt["lo"], tgt["hi"], tgt["ta"], tgt["tb"], tgt["dflt"]
    return e


TGT_ON, TGT_LO, TGT_HI, TGT_DEFAULT, TGT_CAST_SHIFT = 1, 2, 4, 8, 4  # mirrors csrc/common.h
_CASTS = {None: 0, "round": 1, "ceiling": 2, "floor": 3}


def target_post(t, force: bool = False) -> Optional[dict]:
    """The epilogue's PMML Target stage for a regression value (JPMML ``TargetUtil`` order: clip
    to [min, max], then ``* rescaleFactor + rescaleConstant``, then ``castInteger``; a row without
    a prediction takes ``TargetValue defaultValue``). None when the target is a pure rescale that
    the caller folds into the affine map (``force``: always build the stage, e.g. after a link)."""
    if t is None:
        return None
    dflt = t.values[0].default_value if t.values and t.values[0].default_value is not None else None
    if not force and t.min is None and t.max is None and not t.cast_integer and dflt is None:
        return None
    if t.cast_integer not in _CASTS:
        raise NotLowerable(f"Target castInteger {t.cast_integer!r}")
    flags = TGT_ON | (TGT_LO if t.min is not None else 0) | (TGT_HI if t.max is not None else 0) \
        | (TGT_DEFAULT if dflt is not None else 0) | (_CASTS[t.cast_integer] << TGT_CAST_SHIFT)
    return dict(flags=flags, lo=float(t.min) if t.min is not None else 0.0,
                hi=float(t.max) if t.max is not None else 0.0, ta=float(t.rescale_factor),
                tb=float(t.rescale_constant), dflt=float(dflt) if dflt is not None else 0.0)


def apply_target_torch(s, ok, tgt: Optional[dict]):
    """Torch twin of ``apply_target`` in csrc/epilogue.h (host epilogues: split / sharded / GEMM paths)."""
    import torch

    if not tgt:
        return s, ok
    f = tgt["flags"]
    out_dtype = s.dtype
    s = s.double()  # fp64 like csrc/epilogue.h apply_target (and the oracle)
    if f & TGT_LO:
        s = torch.where(s < tgt["lo"], torch.full_like(s, tgt["lo"]), s)
    if f & TGT_HI:
        s = torch.where(s > tgt["hi"], torch.full_like(s, tgt["hi"]), s)
    s = s * tgt["ta"] + tgt["tb"]
    cast = (f >> TGT_CAST_SHIFT) & 3
    if cast == 1:
        s = torch.floor(s + 0.5)
    elif cast == 2:
        s = torch.ceil(s)
    elif cast == 3:
        s = torch.floor(s)
    if f & TGT_DEFAULT:
        s = torch.where(ok, s, torch.full_like(s, tgt["dflt"]))
        ok = torch.ones_like(ok)
    return s.to(out_dtype), ok


def _addr(t) -> Optional[int]:
    """Tensor or raw integer address -> address (None stays NULL)."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _label_table(labels: List[str]) -> np.ndarray:
    out = np.empty(len(labels), dtype=np.float32)
    for i, s in enumerate(labels):
        try:
            out[i] = float(s)
        except (TypeError, ValueError):
            out[i] = np.nan
    return out


# --------------------------------------------------------------------------- clustering


class ClusterPlan(DevicePlan):
    kind = "cluster"
    _STATE = DevicePlan._STATE + ("centers", "weights", "scales", "qweights", "cfun", "table", "metric_code",
                                  "similarity", "p", "variant", "wc", "cc")
    _METRICS = {"squaredEuclidean": 0, "euclidean": 1, "cityBlock": 2, "chebychev": 3, "minkowski": 4}
    _CF = {"absDiff": 0, "gaussSim": 1, "delta": 2, "equal": 3}
    MFMA_MIN_K = 16  # below this the VALU kernel's per-cluster loop is as fast as a 32-wide MFMA tile

    def __init__(self, compiled, device, cluster_variant: str = "auto", **_):
        """``cluster_variant``: ``"valu"`` (exact per-cluster Σ w(x-c)², every metric), ``"mfma"``
        (matrix-core ‖x‖² − 2x·c + ‖c‖², squared / plain Euclidean with absDiff only; rows with
        missing values fall back to the exact form inside the kernel) or ``"auto"`` (MFMA when it
        applies and K ≥ ``MFMA_MIN_K``)."""
        super().__init__(compiled, device)
        ev: ClusteringEvaluator = compiled.evaluator
        if getattr(ev, "knn", None) is not None and (min(ev.k, len(ev.targets)) > 1 or ev.target is not None):
            raise NotLowerable("k-NN with k > 1 or a Target runs on the k-NN kernel (KnnPlan)")
        if ev.metric not in self._METRICS:
            raise NotLowerable(f"clustering metric {ev.metric!r} is host-only")
        if ev.fields != compiled.active_fields:
            raise NotLowerable("clustering fields differ from the active fields (derived inputs are host-only)")
        if not compiled.target_fields:
            raise NotLowerable("clustering model without a target field")
        self.metric_code = self._METRICS[ev.metric]
        self.similarity = 0 if ev.kind_distance else 1
        self.p = float(ev.p)
        self.centers = self._t(ev.centers.astype(np.float32))
        self.weights = self._t(ev.weights.astype(np.float32))
        self.scales = self._t(ev.scales.astype(np.float32))
        self.qweights = self._t(ev.missing_weights.astype(np.float32))
        self.cfun = self._t(np.array([self._CF[c] for c in ev.compare], dtype=np.int32))
        self.table = self._t(_label_table(ev.entity_ids))
        mfma_ok = (self.similarity == 0 and self.metric_code in (0, 1)
                   and all(c == "absDiff" for c in ev.compare) and compiled.n_features <= 128)
        if cluster_variant not in ("auto", "valu", "mfma"):
            raise ValueError(f"cluster_variant {cluster_variant!r}")
        if cluster_variant == "mfma" and not mfma_ok:
            raise NotLowerable("MFMA clustering needs squared/plain euclidean distance with absDiff")
        use = cluster_variant == "mfma" or (cluster_variant == "auto" and mfma_ok
                                            and len(ev.centers) >= self.MFMA_MIN_K)
        self.variant = "mfma" if use else "valu"
        self.wc = self.cc = None
        if use:
            wc, cc = self.mfma_operands(ev.centers, ev.weights)
            self.wc, self.cc = self._t(wc), self._t(cc)

    @staticmethod
    def mfma_operands(centers: np.ndarray, weights: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """``wc [Kp][Fp] = w ∘ c`` zero padded to the 32×2 MFMA tile, ``cc [Kp] = Σ_f w_f c_f²``
        (fp64 sum, +inf on padded clusters so they never win the argmin)."""
        K, F = centers.shape
        Kp, Fp = -(-K // 32) * 32, -(-F // 2) * 2
        wc = np.zeros((Kp, Fp), dtype=np.float32)
        c32 = centers.astype(np.float32).astype(np.float64)
        w32 = weights.astype(np.float32).astype(np.float64)
        wc[:K, :F] = (c32 * w32).astype(np.float32)
        cc = np.full(Kp, np.inf, dtype=np.float32)
        cc[:K] = (c32 * c32 * w32).sum(axis=1).astype(np.float32)
        return wc, cc

    def launch(self, X, score, valid, stream=None, probs=None, label=None, affinity=None) -> None:
        from ..ops._lib import ClusterArgs, check, ptr, stream_handle

        a = ClusterArgs()
        a.X = ptr(X)
        a.n_rows, a.n_feat, a.ldx, a.K = X.shape[0], X.shape[1], X.stride(0), self.centers.shape[0]
        a.prep = ptr(self.prep)
        a.centers, a.weights, a.scales = ptr(self.centers), ptr(self.weights), ptr(self.scales)
        a.qweights, a.cfun, a.table = ptr(self.qweights), ptr(self.cfun), ptr(self.table)
        a.metric, a.similarity, a.p = self.metric_code, self.similarity, self.p
        a.score, a.valid, a.label, a.affinity = ptr(score), ptr(valid), ptr(label), ptr(affinity)
        import ctypes

        if self.variant == "mfma":
            Kp, Fp = self.wc.shape
            check(self.lib.pmml_cluster_mfma_launch(stream_handle(stream), ctypes.byref(a), ptr(self.wc),
                                                    ptr(self.cc), Kp, Fp), "cluster mfma kernel")
        else:
            check(self.lib.pmml_cluster_launch(stream_handle(stream), ctypes.byref(a)), "cluster kernel")


class KnnPlan(DevicePlan):
    """NearestNeighborModel with ``k > 1`` on ``knn.hip``: instance distances (VALU, or MFMA
    expansion for squared / plain euclidean absDiff distances over many instances), a register
    top-k and the PMML aggregation (vote / average / median / weighted forms) in the same kernel.
    Mirrors :class:`~flink_jpmml_amd.models.knn.NearestNeighborEvaluator`; ``k == 1`` stays a
    clustering argmin (:class:`ClusterPlan`)."""

    kind = "knn"
    _STATE = DevicePlan._STATE + ("inst", "weights", "scales", "qweights", "cfun", "inst_value", "inst_class",
                                  "class_table", "metric_code", "similarity", "p", "k", "agg", "threshold",
                                  "variant", "wc", "cc", "tgt")
    _AGG = {"majorityVote": 0, "weightedMajorityVote": 1, "average": 2, "median": 3, "weightedAverage": 4}
    K_MAX = 32
    MFMA_MIN_INSTANCES = 64

    def __init__(self, compiled, device, knn_variant: str = "auto", **_):
        super().__init__(compiled, device)
        ev = compiled.evaluator
        m = ev.knn
        k = min(ev.k, len(ev.targets))
        if k > self.K_MAX:
            raise NotLowerable(f"k-NN with k = {k} > {self.K_MAX} is host-only")
        if ev.metric not in ClusterPlan._METRICS:
            raise NotLowerable(f"k-NN metric {ev.metric!r} is host-only")
        if ev.fields != compiled.active_fields:
            raise NotLowerable("k-NN inputs differ from the active fields (derived inputs are host-only)")
        if compiled.n_features > 128:
            raise NotLowerable("k-NN over more than 128 inputs is host-only")
        method = m.categorical_method if ev.kind == "classification" else m.continuous_method
        if method not in self._AGG or (ev.kind == "classification") != (self._AGG[method] < 2):
            raise NotLowerable(f"k-NN scoring method {method!r} is host-only")
        self.metric_code = ClusterPlan._METRICS[ev.metric]
        self.similarity = 0 if ev.kind_distance else 1
        self.p = float(ev.p)
        self.k = int(k)
        self.agg = self._AGG[method]
        self.threshold = float(m.threshold)
        self.inst = self._t(ev.centers.astype(np.float32))
        self.weights = self._t(ev.weights.astype(np.float32))
        self.scales = self._t(ev.scales.astype(np.float32))
        self.qweights = self._t(ev.missing_weights.astype(np.float32))
        self.cfun = self._t(np.array([ClusterPlan._CF[c] for c in ev.compare], dtype=np.int32))
        if ev.kind == "classification":
            self.inst_class = self._t(np.asarray(ev.inst_class, dtype=np.int32))
            self.class_table = self._t(_label_table(ev.categories))
            self.inst_value = None
            self.tgt = None
        else:
            self.inst_value = self._t(ev.inst_value.astype(np.float32))
            self.inst_class = self.class_table = None
            self.tgt = target_post(ev.target, force=True) if ev.target is not None else None
        mfma_ok = (self.similarity == 0 and self.metric_code in (0, 1) and all(c == "absDiff" for c in ev.compare))
        if knn_variant not in ("auto", "valu", "mfma"):
            raise ValueError(f"knn_variant {knn_variant!r}")
        if knn_variant == "mfma" and not mfma_ok:
            raise NotLowerable("MFMA k-NN needs squared/plain euclidean distance with absDiff")
        use = knn_variant == "mfma" or (knn_variant == "auto" and mfma_ok
                                        and len(ev.centers) >= self.MFMA_MIN_INSTANCES)
        self.variant = "mfma" if use else "valu"
        self.wc = self.cc = None
        if use:
            wc, cc = ClusterPlan.mfma_operands(ev.centers, ev.weights)
            self.wc, self.cc = self._t(wc), self._t(cc)

    def launch(self, X, score, valid, stream=None, probs=None) -> None:
        import ctypes

        from ..ops._lib import KnnArgs, check, ptr, stream_handle

        a = KnnArgs()
        a.X = ptr(X)
        a.n_rows, a.n_feat, a.ldx, a.n_inst = X.shape[0], X.shape[1], X.stride(0), self.inst.shape[0]
        a.prep = ptr(self.prep)
        a.inst, a.weights, a.scales, a.qweights = ptr(self.inst), ptr(self.weights), ptr(self.scales), ptr(self.qweights)
        a.cfun, a.inst_value, a.inst_class = ptr(self.cfun), ptr(self.inst_value), ptr(self.inst_class)
        a.class_table = ptr(self.class_table)
        a.metric, a.similarity, a.p, a.k = self.metric_code, self.similarity, self.p, self.k
        a.agg, a.threshold = self.agg, self.threshold
        a.epi = _epilogue(0, tgt=self.tgt)
        a.score, a.valid = ptr(score), ptr(valid)
        if self.variant == "mfma":
            Np, Fp = self.wc.shape
            check(self.lib.pmml_knn_launch(stream_handle(stream), ctypes.byref(a), ptr(self.wc), ptr(self.cc),
                                           Np, Fp), "k-NN mfma kernel")
        else:
            check(self.lib.pmml_knn_launch(stream_handle(stream), ctypes.byref(a), None, None, 0, 0), "k-NN kernel")


# --------------------------------------------------------------------------- linear


class LinearPlan(DevicePlan):
    kind = "linear"
    _STATE = DevicePlan._STATE + ("W", "b", "K", "simplemax", "table", "epi_args")

    def __init__(self, compiled, device):
        super().__init__(compiled, device)
        ev: RegressionEvaluator = compiled.evaluator
        if not ev.is_dense_linear():
            raise NotLowerable("regression tables with categorical predictors / terms are host-only")
        if ev.numeric_fields != compiled.active_fields[: len(ev.numeric_fields)] or \
                set(ev.numeric_fields) != set(compiled.active_fields):
            # reorder W rows to the active-field order
            pass
        W, b = ev.dense_weights()
        Wf = np.zeros((compiled.n_features, W.shape[1]))
        for i, name in enumerate(ev.numeric_fields):
            if name not in compiled.active_fields:
                raise NotLowerable(f"predictor {name!r} is not an active field")
            Wf[compiled.active_fields.index(name)] = W[i]
        self.used = np.zeros(compiled.n_features, dtype=bool)
        for name in ev.numeric_fields:
            self.used[compiled.active_fields.index(name)] = True
        if not self.used.all():
            raise NotLowerable("unused active fields would wrongly invalidate rows with missing values")
        self.W = self._t(Wf.astype(np.float32))
        self.b = self._t(b.astype(np.float32))
        self.K = W.shape[1]
        norm = ev.rm.normalization_method
        self.simplemax = 0
        if ev.kind == "classification":
            self.table = self._t(_label_table(ev.categories))
            if norm == "softmax":
                self.epi_args = dict(mode=EPI_SOFTMAX, C=self.K)
            elif norm == "simplemax":
                self.simplemax = 1
                self.epi_args = dict(mode=EPI_ARGMAX, C=self.K)
            elif norm.startswith("cumulative:"):  # ordinal GLM (runtime/design.py)
                lk = norm.split(":", 1)[1]
                if lk not in LINKS or lk in ("none", "exp"):
                    raise NotLowerable(f"cumulativeLink {lk!r}")
                self.epi_args = dict(mode=EPI_CUMULATIVE, C=self.K, link=LINKS[lk])
            elif self.K == 2:
                if norm not in LINKS:
                    raise NotLowerable(f"normalizationMethod {norm!r}")
                # p0 = link(y0); the second table is ignored (PMML binary rule)
                self.epi_args = dict(mode=EPI_LOGISTIC2, C=2, link=LINKS[norm])
            else:  # > 2 tables: every class its own link value, first argmax (models/regression.py)
                if norm not in LINKS:
                    raise NotLowerable(f"normalizationMethod {norm!r}")
                self.epi_args = dict(mode=EPI_LINKMAX, C=self.K, link=LINKS[norm])
        else:
            self.table = None
            if norm not in LINKS:
                raise NotLowerable(f"normalizationMethod {norm!r}")
            tgt = ev.target
            self.epi_args = dict(mode=EPI_AFFINE, link=LINKS[norm])
            post = target_post(tgt, force=norm not in ("none", None))  # rescale after a link: Target stage
            if post is not None:
                self.epi_args["tgt"] = post
            elif tgt is not None:
                self.epi_args.update(a=tgt.rescale_factor, b=tgt.rescale_constant)  # folded

    supports_direct = True

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None) -> None:
        import ctypes

        from ..ops._lib import LinearArgs, check, ptr, stream_handle

        a = LinearArgs()
        a.X = ptr(X)
        a.n_rows, a.n_feat, a.ldx, a.K = X.shape[0], X.shape[1], X.stride(0), self.K
        a.prep, a.W, a.bias, a.simplemax = ptr(self.prep), ptr(self.W), ptr(self.b), self.simplemax
        a.epi = _epilogue(table=self.table, write_probs=probs is not None, **self.epi_args)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.probs = _addr(score), _addr(valid), ptr(probs)
        check(self.lib.pmml_linear_launch(stream_handle(stream), ctypes.byref(a)), "linear kernel")


# --------------------------------------------------------------------------- tree ensembles


@dataclass
class EnsembleSpec:
    trees: List[BinaryTree]
    weights: List[float]
    P: int  # leaf payload width
    C: int  # accumulator slots
    epi: dict
    labels: Optional[List[str]]
    slots: Optional[List[int]] = None
    mode: str = "sum"  # sum | slot (multi-class chains) | class (majority vote: leaf = class index)
    tree_w: Optional[List[float]] = None  # mode "class": per-tree vote weight
    acc_init: Optional[List[float]] = None  # multi-class: per-class initial accumulator


def to_general(spec: "EnsembleSpec") -> "EnsembleSpec":
    """The same ensemble in the P=C payload form the narrow / pointer kernels accumulate in LDS:
    votes become weighted one-hot leaves, per-class biases become constant stump trees."""
    if spec.mode == "sum":
        return spec
    if spec.mode == "class":
        trees = []
        for t, w in zip(spec.trees, spec.tree_w or [1.0] * len(spec.trees)):
            probs = np.zeros((len(t.leaf_value), spec.C))
            ok = ~np.isnan(t.leaf_value)
            probs[np.nonzero(ok)[0], t.leaf_value[ok].astype(int)] = w
            trees.append(dataclasses.replace(t, leaf_probs=probs))
        return EnsembleSpec(trees, [1.0] * len(trees), spec.C, spec.C, spec.epi, spec.labels)
    # slot: one payload value per tree into its class slot; biases as constant stumps
    trees, weights, slots = list(spec.trees), list(spec.weights), list(spec.slots)
    for k, b in enumerate(spec.acc_init or []):
        if b != 0.0:
            trees.append(_stump(b))
            weights.append(1.0)
            slots.append(k)
    return EnsembleSpec(trees, weights, 1, spec.C, spec.epi, spec.labels, slots)


def _stump(value: float) -> BinaryTree:
    """A single-leaf tree scoring ``value`` for every row."""
    return BinaryTree(feature=np.array([-1]), threshold=np.zeros(1), op=np.zeros(1, dtype=np.int64),
                      left=np.array([-1]), right=np.array([-1]), default_left=np.zeros(1, dtype=bool),
                      leaf_value=np.array([float(value)]), leaf_probs=None, depth=0, null_missing=False)


def _segments_all_true(mm: ir.MiningModel) -> bool:
    return all(isinstance(s.predicate, ir.TruePredicate) for s in mm.segments)


def _target_affine(ev, allow_post: bool = False) -> Tuple[float, float]:
    """The target's rescale as an affine map folded into the ensemble epilogue; with a clip / cast /
    default stage (:func:`target_post`) the rescale moves into that stage (``allow_post``: only at
    the top level, where the epilogue applies it) and the affine map is the identity."""
    t = ev.target
    if t is None:
        return 1.0, 0.0
    if target_post(t) is not None:
        if not allow_post:
            raise NotLowerable("nested Target min/max/castInteger/defaultValue is host-only")
        return 1.0, 0.0
    return t.rescale_factor, t.rescale_constant


def _regression_ensemble(ev, field_index, lower=lower_binary_tree,
                         allow_post: bool = False) -> Tuple[List[BinaryTree], List[float], float, float]:
    """Flatten a regression tree / MiningModel(sum|average|weightedAverage) of regression trees
    into (trees, per-tree weights, a, b) with value = a * Σ w_t leaf_t + b."""
    if isinstance(ev, TreeEvaluator):
        if ev.kind != "regression":
            raise NotLowerable("expected a regression tree")
        a, b = _target_affine(ev, allow_post)
        return [lower(ev, field_index)], [1.0], a, b
    if isinstance(ev, MiningEvaluator):
        mm = ev.mm
        if ev.kind != "regression":
            raise NotLowerable("expected a regression ensemble")
        if not _segments_all_true(mm):
            raise NotLowerable("segment predicates other than True are host-only")
        method = mm.multiple_model_method
        if method not in ("sum", "weightedSum", "average", "weightedAverage"):
            raise NotLowerable(f"multipleModelMethod {method!r} is host-only for regression ensembles")
        trees: List[BinaryTree] = []
        weights: List[float] = []
        for seg, sub in zip(mm.segments, ev.sub):
            st, sw, sa, sb = _regression_ensemble(sub, field_index, lower)
            if sb != 0.0:
                raise NotLowerable("nested Target rescaleConstant inside an ensemble is host-only")
            w = seg.weight if method in ("weightedAverage", "weightedSum") else 1.0
            trees.extend(st)
            weights.extend([x * w * sa for x in sw])
        _check_null_trees(mm, trees)
        if method == "average":
            scale = 1.0 / max(1, len(mm.segments))
        elif method == "weightedAverage":
            scale = 1.0 / sum(s.weight for s in mm.segments)
        else:
            scale = 1.0
        a, b = _target_affine(ev, allow_post)
        return trees, weights, a * scale, b
    raise NotLowerable(f"{type(ev).__name__} is not a regression tree ensemble")


def _check_null_trees(mm: ir.MiningModel, trees: List[BinaryTree]) -> None:
    """A null tree poisons the row (the ``returnMissing``/``continue`` rule); ``skipSegment``
    would need it dropped from the aggregate instead."""
    if mm.missing_prediction_treatment == "skipSegment" and any(t.null_missing for t in trees):
        raise NotLowerable("skipSegment over null-on-missing trees is host-only")


class NotBinaryForm(NotLowerable):
    """A tree is not in binary-split form: only the GENERAL (predicate-VM) layout can score it."""


def ensemble_spec(compiled, lower=lower_binary_tree) -> EnsembleSpec:
    ev = compiled.evaluator
    field_index = getattr(compiled, "field_index", None) or {f: i for i, f in enumerate(compiled.active_fields)}
    try:
        if ev.kind == "regression":
            trees, w, a, b = _regression_ensemble(ev, field_index, lower, allow_post=True)
            epi = dict(mode=EPI_AFFINE, a=a, b=b)
            post = target_post(ev.target)
            if post is not None:
                epi["tgt"] = post
            return EnsembleSpec(trees, w, 1, 1, epi, None)
        if isinstance(ev, MiningEvaluator) and ev.mm.multiple_model_method == "modelChain":
            return _chain_spec(compiled, ev, field_index, lower)
        if isinstance(ev, MiningEvaluator) and ev.kind == "classification":
            return _classification_spec(ev, field_index, lower)
        if isinstance(ev, TreeEvaluator) and ev.kind == "classification":
            t = lower(ev, field_index)
            C = len(ev.categories)
            return EnsembleSpec([t], [1.0], C, C, dict(mode=EPI_ARGMAX, C=C, a=1.0), list(ev.categories))
    except NotBinary as e:
        raise NotBinaryForm(f"tree is not in binary-split form: {e}") from e
    raise NotLowerable(f"{type(ev).__name__} ({ev.kind}) is not a lowerable tree ensemble")


def _classification_spec(ev: MiningEvaluator, field_index, lower=lower_binary_tree) -> EnsembleSpec:
    mm = ev.mm
    if not _segments_all_true(mm):
        raise NotLowerable("segment predicates other than True are host-only")
    method = mm.multiple_model_method
    cats = list(ev.categories)
    C = len(cats)
    trees, weights = [], []
    vote = method in ("majorityVote", "weightedMajorityVote")
    for seg, sub in zip(mm.segments, ev.sub):
        if not isinstance(sub, TreeEvaluator) or sub.kind != "classification":
            raise NotLowerable("classification ensembles must hold classification trees")
        t = lower(sub, field_index)
        remap = np.array([cats.index(c) for c in sub.categories])
        if vote:
            # the leaf is the (ensemble-order) class index; the tree's weight is its vote
            ok = ~np.isnan(t.leaf_value)
            lv = np.full(len(t.leaf_value), np.nan)
            lv[ok] = remap[t.leaf_value[ok].astype(int)]
            t.leaf_value = lv
        elif method in ("average", "weightedAverage"):
            probs = np.zeros((len(t.leaf_value), C))
            probs[:, remap] = np.nan_to_num(t.leaf_probs)
            t.leaf_probs = probs
        else:
            raise NotLowerable(f"multipleModelMethod {method!r} is host-only for classification")
        trees.append(t)
        weights.append(seg.weight if method.startswith("weighted") else 1.0)
    _check_null_trees(mm, trees)
    epi = dict(mode=EPI_ARGMAX, C=C, a=1.0 / sum(weights))
    if vote:
        return EnsembleSpec(trees, [1.0] * len(trees), 1, C, epi, cats, mode="class", tree_w=weights)
    return EnsembleSpec(trees, weights, C, C, epi, cats)


def _chain_spec(compiled, ev: MiningEvaluator, field_index, lower=lower_binary_tree) -> EnsembleSpec:
    """modelChain [regression tree ensemble(s) -> classification RegressionModel on their outputs]
    fused into one kernel + epilogue: the XGBoost / LightGBM binary export (one ensemble + logistic
    calibrator) and the K-class export (K ensembles, one per class, + softmax RegressionModel)."""
    mm = ev.mm
    if len(mm.segments) < 2 or not _segments_all_true(mm):
        raise NotLowerable("modelChain needs >= 2 segments with True predicates")
    *firsts, second = ev.sub
    if not isinstance(second, RegressionEvaluator) or second.kind != "classification":
        raise NotLowerable("chain calibrator must be a classification RegressionModel")
    outs = {}  # output field -> ensemble index
    for i, first in enumerate(firsts):
        o = [o for o in first.model.output if o.feature in ("predictedValue", "transformedValue")
             and o.expression is None]
        if len(o) < 1:
            raise NotLowerable("chain segment exposes no predictedValue output")
        outs[o[0].name] = i
    rm = second.rm
    norm = rm.normalization_method
    cats = list(second.categories)
    if len(firsts) == 1:
        out_name = next(iter(outs))
        if len(rm.tables) != 2 or rm.tables[1].numeric or rm.tables[1].categorical or rm.tables[1].terms:
            raise NotLowerable("calibrator must have two tables, the second constant")
        t0 = rm.tables[0]
        if t0.categorical or t0.terms or len(t0.numeric) != 1 or t0.numeric[0].name != out_name \
                or t0.numeric[0].exponent != 1.0:
            raise NotLowerable("calibrator must be linear in the ensemble output")
        if norm not in LINKS or norm == "none":
            raise NotLowerable(f"calibrator normalizationMethod {norm!r} is host-only")
        trees, w, a, b = _regression_ensemble(firsts[0], field_index, lower)
        coef, icpt = t0.numeric[0].coefficient, t0.intercept
        # the chain's target is the calibrator's; category table in calibrator order
        return EnsembleSpec(trees, w, 1, 1, dict(mode=EPI_LOGISTIC2, C=2, a=coef * a, b=coef * b + icpt,
                                                 link=LINKS[norm]), cats)
    # K-class: table k = intercept_k + coef_k * output(ensemble e_k); softmax over the K tables
    if norm != "softmax":
        raise NotLowerable(f"K-class chain normalizationMethod {norm!r} is host-only (softmax only)")
    K = len(rm.tables)
    if K < 2 or K > 16:
        raise NotLowerable(f"K-class chains with {K} classes are host-only (2..16)")
    trees, weights, slots, init = [], [], [], []
    for k, tab in enumerate(rm.tables):
        if tab.categorical or tab.terms or len(tab.numeric) > 1:
            raise NotLowerable("K-class calibrator tables must be linear in one ensemble output")
        if not tab.numeric:
            init.append(tab.intercept)
            continue
        p = tab.numeric[0]
        if p.exponent != 1.0 or p.name not in outs:
            raise NotLowerable("K-class calibrator tables must reference a chain output linearly")
        et, ew, ea, eb = _regression_ensemble(firsts[outs[p.name]], field_index, lower)
        trees.extend(et)
        weights.extend(x * ea * p.coefficient for x in ew)
        slots.extend([k] * len(et))
        init.append(tab.intercept + p.coefficient * eb)
    return EnsembleSpec(trees, weights, 1, K, dict(mode=EPI_SOFTMAX, C=K, a=1.0), cats, slots=slots, mode="slot",
                        acc_init=init)


def shard_spec(spec: EnsembleSpec, rank: int, world: int) -> EnsembleSpec:
    """Rank ``rank``'s contiguous slice of a single-accumulator ensemble with a raw epilogue
    (``mode=AFFINE, a=1, b=0``, no link): the kernel writes ``Σ w_i·leaf_i`` over its trees, or
    NaN/invalid for rows a null-on-missing tree poisons."""
    if spec.P != 1 or spec.mode != "sum" or spec.epi["mode"] not in (EPI_AFFINE, EPI_LOGISTIC2):
        raise NotLowerable("tree sharding supports single-score ensembles (regression / binary chains)")
    if not 0 <= rank < world or len(spec.trees) < world:
        raise ValueError(f"cannot shard {len(spec.trees)} trees over {world} ranks (rank {rank})")
    base, rem = divmod(len(spec.trees), world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return EnsembleSpec(spec.trees[lo:hi], spec.weights[lo:hi], 1, 1, dict(mode=EPI_AFFINE, a=1.0, b=0.0),
                        None, spec.slots[lo:hi] if spec.slots is not None else None)


def _perfect_pack(trees: List[BinaryTree], weights: List[float], P: int, D: int, stride: int = TB,
                  fmap: Optional[dict] = None, leaf_bits: Optional[str] = None) -> Tuple[np.ndarray, int, bool]:
    """Pack trees into the PERFECT layout (heap order, root = node 1):

    ``[ (2^D-1) x {T bits, feature byte offset} ][ 2^D x P leaves ][ ceil((2^D-1)/32) default-right words ]``

    padded to 16 bytes. Split tests are canonicalised to "go right iff x >= T"
    (:func:`canonical_threshold`); a missing value goes right iff the node's default-right bit is
    set. Leaves above depth D are replicated over their whole padded subtree.

    The feature byte offset is ``column * stride * 4`` with ``column = fmap[feature]`` (the
    kernel's staged-column order) and ``stride`` its feature-plane stride in floats (``TB`` for
    the narrow kernel, ``rows`` for the wide one). ``leaf_bits="vote8"`` stores the packed
    vote increment ``1 << 8*class`` as the leaf's bit pattern (class-index leaves)."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    rec = 2 * NI + NL * P + ndr
    rec = (rec + 3) & ~3
    if trees and (P == 1 or all(t.leaf_probs is not None for t in trees)):
        return _perfect_pack_vec(trees, weights, P, D, stride, fmap, leaf_bits, rec)
    return _perfect_pack_loop(trees, weights, P, D, stride, fmap, leaf_bits, rec)


def _perfect_pack_loop(trees, weights, P: int, D: int, stride: int, fmap, leaf_bits, rec: int):
    """Per-node reference implementation of :func:`_perfect_pack` (the vectorised packer is
    tested bit-identical against it)."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    blob = np.zeros((len(trees), rec), dtype=np.uint32)
    has_dr = False
    for ti, (t, w) in enumerate(zip(trees, weights)):
        nodes_T = np.zeros(NI, dtype=np.float32)
        nodes_meta = np.zeros(NI, dtype=np.uint32)
        leaves = np.zeros((NL, P), dtype=np.float32)
        dr_bits = np.zeros(ndr * 32, dtype=np.uint32)
        stack = [(0, 0, 0, None)]  # (node k, level-order index p, depth, parent split's meta)
        while stack:
            k, p, d, pm = stack.pop()
            if t.feature[k] < 0:
                # the padded nodes below a leaf above depth D read the parent split's column: the
                # walk visited it already, so a NaN there cannot newly null a nullPrediction tree
                # (column 0 could be missing when the path never touched it)
                if pm is not None:
                    q, cnt = p, 1
                    while q < NI:
                        nodes_meta[q: min(q + cnt, NI)] = pm
                        q, cnt = 2 * q + 1, 2 * cnt
                if leaf_bits == "vote8":
                    val = np.array([np.uint32(1 << (8 * int(t.leaf_value[k]))).view(np.float32)])
                else:
                    val = (t.leaf_probs[k] if t.leaf_probs is not None and P > 1 else np.array([t.leaf_value[k]])) * w
                lo = p
                for _ in range(D - d):
                    lo = 2 * lo + 1
                span = 1 << (D - d)
                if leaf_bits == "vote8":
                    leaves[lo - NI: lo - NI + span, :] = val[None, :P]
                else:
                    leaves[lo - NI: lo - NI + span, :] = np.asarray(val, dtype=np.float64)[None, :P]
                continue
            T, swap = canonical_threshold(int(t.op[k]), float(t.threshold[k]))
            first, second = int(t.left[k]), int(t.right[k])
            dflt_first = bool(t.default_left[k])
            if swap:
                left_child, right_child = second, first
                dr = dflt_first  # default went to the (now right) first child
            else:
                left_child, right_child = first, second
                dr = not dflt_first
            f = int(t.feature[k]) if fmap is None else fmap[int(t.feature[k])]
            if stride == TB and f > 63:
                raise NotLowerable("the narrow perfect layout supports at most 64 features")
            nodes_T[p] = T
            nodes_meta[p] = f * stride * 4
            if dr:
                dr_bits[p] = 1
                has_dr = True
            stack.append((left_child, 2 * p + 1, d + 1, nodes_meta[p]))
            stack.append((right_child, 2 * p + 2, d + 1, nodes_meta[p]))
        if t.null_missing and t.feature[0] >= 0:
            dr_bits[NI] = 1  # tree-level null-on-missing flag (node index NI does not exist)
        blob[ti, 0: 2 * NI: 2] = nodes_T.view(np.uint32)
        blob[ti, 1: 2 * NI: 2] = nodes_meta
        blob[ti, 2 * NI: 2 * NI + NL * P] = leaves.reshape(-1).view(np.uint32)
        words = (dr_bits.reshape(ndr, 32) << np.arange(32, dtype=np.uint32)[None, :]).sum(axis=1, dtype=np.uint64)
        blob[ti, 2 * NI + NL * P: 2 * NI + NL * P + ndr] = words.astype(np.uint32)
    return blob, rec, has_dr


def _canonical_vec(op: np.ndarray, t: np.ndarray):
    """:func:`canonical_threshold` over arrays: ``(T, swap)``."""
    t32 = t.astype(np.float32)
    back = t32.astype(np.float64)
    ceil32 = np.where(back < t, np.nextafter(t32, np.float32(np.inf)), t32)     # smallest fp32 >= t
    floor32 = np.where(back > t, np.nextafter(t32, np.float32(-np.inf)), t32)   # largest fp32 <= t
    up_floor = np.nextafter(floor32, np.float32(np.inf))
    T = np.where((op == OP_LT) | (op == OP_GE), ceil32, up_floor)
    swap = (op == OP_GT) | (op == OP_GE)
    return T.astype(np.float32), swap


def _perfect_pack_vec(trees, weights, P: int, D: int, stride: int, fmap, leaf_bits, rec: int):
    """Vectorised :func:`_perfect_pack` (bit-identical): all trees advance one heap level at a
    time over concatenated node arrays — no per-node Python loop (model load time)."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    n = len(trees)
    sizes = np.array([len(t.feature) for t in trees], np.int64)
    off = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    feat = np.concatenate([t.feature for t in trees]).astype(np.int64)
    thr = np.concatenate([t.threshold for t in trees]).astype(np.float64)
    ops = np.concatenate([t.op for t in trees])
    dleft = np.concatenate([t.default_left for t in trees])
    tree_of = np.repeat(np.arange(n), sizes)
    left = np.concatenate([t.left for t in trees]).astype(np.int64) + off[tree_of]
    right = np.concatenate([t.right for t in trees]).astype(np.int64) + off[tree_of]
    w_node = np.asarray(weights, np.float64)[tree_of]
    T, swap = _canonical_vec(ops, thr)
    lc = np.where(swap, right, left)
    rc = np.where(swap, left, right)
    dr = np.where(swap, dleft, ~dleft)
    if fmap is None:
        col = feat
    else:
        lut = np.full(max(fmap) + 1 if fmap else 1, -1, np.int64)
        for k, v in fmap.items():
            lut[k] = v
        col = np.where(feat >= 0, lut[np.clip(feat, 0, len(lut) - 1)], -1)
    if stride == TB and (col[feat >= 0] > 63).any():
        raise NotLowerable("the narrow perfect layout supports at most 64 features")
    nodes_T = np.zeros((n, NI), np.float32)
    nodes_meta = np.zeros((n, NI), np.uint32)
    dr_bits = np.zeros((n, ndr * 32), np.uint32)
    cur = off.copy()[:, None]  # [n, 1] node at each heap position of the current level
    pm = np.full((n, 1), -1, np.int64)  # meta of the deepest real split above (-1: none)
    for d in range(D):
        split = feat[cur] >= 0
        p0 = (1 << d) - 1
        sl = slice(p0, p0 + (1 << d))
        nodes_T[:, sl] = np.where(split, T[cur], 0.0)
        # padded nodes (below a leaf above depth D) read the parent split's column, which the walk
        # visited already: a NaN in a column the path never touched must not null the tree
        meta = np.where(split, col[cur] * stride * 4, np.maximum(pm, 0))
        nodes_meta[:, sl] = meta.astype(np.uint32)
        dr_bits[:, sl] = np.where(split, dr[cur], False)
        # a leaf above depth D covers its whole padded subtree: both "children" are itself
        nxt = np.empty((n, 2 << d), np.int64)
        nxt[:, 0::2] = np.where(split, lc[cur], cur)
        nxt[:, 1::2] = np.where(split, rc[cur], cur)
        cur = nxt
        pm = np.repeat(np.where(split, meta, pm), 2, axis=1)
    if (feat[cur] >= 0).any():
        raise NotLowerable("tree deeper than the PERFECT depth")
    if leaf_bits == "vote8":
        lv = np.concatenate([t.leaf_value for t in trees])
        leaves = (np.uint32(1) << (np.uint32(8) * lv[cur].astype(np.uint32))).view(np.float32)[..., None]
    elif P > 1:
        probs = np.concatenate([t.leaf_probs for t in trees])
        leaves = (probs[cur][..., :P] * w_node[cur][..., None]).astype(np.float32)
    else:
        lv = np.concatenate([t.leaf_value for t in trees])
        leaves = (lv[cur] * w_node[cur]).astype(np.float32)[..., None]
    has_dr = bool(dr_bits.any())
    for ti, t in enumerate(trees):
        if t.null_missing and t.feature[0] >= 0:  # a single-leaf tree never visits a split
            dr_bits[ti, NI] = 1
    blob = np.zeros((n, rec), dtype=np.uint32)
    blob[:, 0:2 * NI:2] = nodes_T.view(np.uint32)
    blob[:, 1:2 * NI:2] = nodes_meta
    blob[:, 2 * NI:2 * NI + NL * P] = np.ascontiguousarray(leaves).reshape(n, NL * P).view(np.uint32)
    words = (dr_bits.reshape(n, ndr, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(axis=2)
    blob[:, 2 * NI + NL * P: 2 * NI + NL * P + ndr] = words.astype(np.uint32)
    return blob, rec, has_dr


VAR_NAN_FAST, VAR_NAN_PLANES, VAR_POINTER_REFILL, VAR_POINTER_COMPACT, VAR_POINTER_MASKED = 4, 8, 16, 32, 64  # tree_common.h
VAR_POINTER_SUPER = 128
VAR_POINTER_USKIP = 256
VAR_POINTER_PEEL = 512
VAR_POINTER_RANK3 = 1024
VAR_POINTER_LDS = 2048  # compact slots walked out of LDS chunks (tree_lds.hip); host-side flag only
VAR_POINTER_INLINE = 4096  # lock-step pointer walk, leaf payloads inline in the parent nodes
VAR_POINTER_LTOP = 8192  # lock-step pointer walk, BFS: levels 0-4 of each group's trees staged in LDS
POINTER_LTOP_NODES = 31  # ... 2^5 - 1 nodes a tree (tree.hip launcher: LTOP 5)
DYN_B, DYN_SLOTS = 8, 16  # csrc: MODE_SUM trees per claimed batch, batch slots per chunk


def _nan_planes(blob: np.ndarray, D: int, F: int, stride: int = TB) -> np.ndarray:
    """Point every default-right node of a P=1 PERFECT blob at the second feature plane (the
    wide kernel stages it with NaN -> +inf): ``x >= T`` then sends a missing value right at those
    nodes and left (NaN compares false) everywhere else — the default direction costs nothing
    per node, so tiles with missing values keep the fast traversal."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    out = blob.copy()
    words = out[:, 2 * NI + NL: 2 * NI + NL + ndr]
    for p in range(NI):
        dr = ((words[:, p >> 5] >> np.uint32(p & 31)) & np.uint32(1)).astype(bool)
        out[dr, 2 * p + 1] += np.uint32(F * stride * 4)
    return out


FP8_MAX = 448.0  # largest finite OCP e4m3fn value


def quantize_fp8(values: np.ndarray, scale: float) -> np.ndarray:
    """fp32 -> OCP e4m3fn bytes of ``values / scale`` (round to nearest even, saturating)."""
    import torch

    v = np.clip(np.asarray(values, np.float64) / scale, -FP8_MAX, FP8_MAX).astype(np.float32)
    return torch.from_numpy(v).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def dequantize_fp8(q: np.ndarray) -> np.ndarray:
    import torch

    return torch.from_numpy(np.ascontiguousarray(q, dtype=np.uint8)).view(torch.float8_e4m3fn).float().numpy()


def _leaf8_pack(blob: np.ndarray, D: int, scale: Optional[float] = None) -> Tuple[np.ndarray, int, float]:
    """Re-pack a P=1 PERFECT blob with fp8 leaves: the two e4m3 leaves under every last-level node
    go into bits [31:16] of that node's meta (left in [23:16], right in [31:24]); one global
    scale (max |leaf| -> 448) is returned for the epilogue. Record: nodes + default-right words."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    leaves = blob[:, 2 * NI: 2 * NI + NL].view(np.float32)
    if scale is None:
        amax = float(np.max(np.abs(leaves))) if leaves.size else 0.0
        scale = amax / FP8_MAX if amax > 0 else 1.0
    q = quantize_fp8(leaves, scale).astype(np.uint32)  # [trees, NL]
    rec = (2 * NI + ndr + 3) & ~3
    out = np.zeros((blob.shape[0], rec), dtype=np.uint32)
    out[:, : 2 * NI] = blob[:, : 2 * NI]
    out[:, 2 * NI: 2 * NI + ndr] = blob[:, 2 * NI + NL: 2 * NI + NL + ndr]
    first_last = NL // 2 - 1  # level-order index of the first last-level node
    for p in range(first_last, NI):
        left, right = 2 * p + 1 - NI, 2 * p + 2 - NI
        meta = out[:, 2 * p + 1]
        if np.any(meta >> 16):
            raise NotLowerable("feature byte offset does not fit the fp8 leaf-pair meta")
        out[:, 2 * p + 1] = meta | (q[:, left] << 16) | (q[:, right] << 24)
    return out, rec, scale


def _vote_codes_pack(blob: np.ndarray, D: int) -> Tuple[np.ndarray, int]:
    """Re-pack a VOTE8 PERFECT blob (leaves = packed-vote increments ``1 << 8*class``) with the
    class index of the two leaves under every last-level node in bits [23:16] / [31:24] of that
    node's meta, like :func:`_leaf8_pack`: no leaf array (a depth-8 record shrinks 3104 -> 2080
    bytes: larger LDS chunks) and no leaf-pair read at the last level."""
    NI, NL = (1 << D) - 1, 1 << D
    ndr = (NI + 31) // 32
    inc = blob[:, 2 * NI: 2 * NI + NL]
    cls = np.zeros_like(inc)
    for k in range(1, 4):
        cls[inc == np.uint32(1 << (8 * k))] = k
    if not np.isin(inc, [np.uint32(1 << (8 * k)) for k in range(4)]).all():
        raise NotLowerable("vote leaves are not single-class increments")
    rec = (2 * NI + ndr + 3) & ~3
    out = np.zeros((blob.shape[0], rec), dtype=np.uint32)
    out[:, : 2 * NI] = blob[:, : 2 * NI]
    out[:, 2 * NI: 2 * NI + ndr] = blob[:, 2 * NI + NL: 2 * NI + NL + ndr]
    for p in range(NL // 2 - 1, NI):
        left, right = 2 * p + 1 - NI, 2 * p + 2 - NI
        meta = out[:, 2 * p + 1]
        if np.any(meta >> 16):
            raise NotLowerable("feature byte offset does not fit the class-code meta")
        out[:, 2 * p + 1] = meta | (cls[:, left] << 16) | (cls[:, right] << 24)
    return out, rec


def _pointer_pack(trees: List[BinaryTree], weights: List[float], P: int):
    nodes: List[Tuple[int, int, int, int]] = []
    leaves: List[np.ndarray] = []
    roots: List[int] = []
    has_dr = False
    for t, w in zip(trees, weights):
        base_map = {}
        order = []
        stack = [0]
        while stack:
            k = stack.pop()
            order.append(k)
            if t.feature[k] >= 0:
                stack.append(int(t.right[k]))
                stack.append(int(t.left[k]))
        for k in order:
            if t.feature[k] < 0:
                val = t.leaf_probs[k] if t.leaf_probs is not None and P > 1 else np.array([t.leaf_value[k]])
                base_map[k] = ~len(leaves)
                leaves.append(np.asarray(val, dtype=np.float64)[:P] * w)
            else:
                base_map[k] = len(nodes)
                nodes.append((0, 0, 0, 0))
        for k in order:
            if t.feature[k] < 0:
                continue
            T, swap = canonical_threshold(int(t.op[k]), float(t.threshold[k]))
            first, second = int(t.left[k]), int(t.right[k])
            dflt_first = bool(t.default_left[k])
            if swap:
                lc, rc, dr = second, first, dflt_first
            else:
                lc, rc, dr = first, second, not dflt_first
            f = int(t.feature[k])
            meta = (f * TB * 4 if f < 64 else f) | ((1 << 31) if dr else 0) | ((1 << 30) if t.null_missing else 0)
            has_dr = has_dr or dr
            nodes[base_map[k]] = (int(np.float32(T).view(np.uint32)), meta, base_map[lc], base_map[rc])
        roots.append(base_map[0])
    nd = np.array(nodes, dtype=np.int64).astype(np.uint32) if nodes else np.zeros((1, 4), np.uint32)
    lv = np.stack(leaves).astype(np.float32) if leaves else np.zeros((1, P), np.float32)
    return nd, lv, np.array(roots, dtype=np.int32), has_dr


# XCD-aware tree slicing of pointer / hybrid forests (csrc tree_block): one slice per XCD
XCD_SLICES = 8


class TreePlan(DevicePlan):
    """GBDT / random forest / single tree / calibrated chain on the HIP traversal kernel."""

    kind = "tree"
    _STATE = DevicePlan._STATE + ("depth", "n_trees", "layout", "P", "C", "general", "rec_words", "chunk_trees",
                                  "blob", "leaves", "roots", "has_dr", "table", "slots", "splits", "epi_args",
                                  "variant", "children", "preds", "pool", "trees_tab", "max_steps", "blob_nan",
                                  "chunk_trees_nan", "full_epi", "labels", "mode", "tree_w", "acc_init", "feat_map",
                                  "rows_wide", "n_stage", "heads", "head_depth", "pointer_ilp", "xcd_split",
                                  "tail_format", "rank_thr", "rank_cnt", "rank_stride", "lds_chunks", "lds_slices",
                                  "lds_rows", "lds_chunk_u4", "lds_n_slices", "mix_mass", "mix_w", "mix_tab",
                                  "mix_remap", "vcol", "leaf_onehot")

    # GENERAL-layout extras (sibling mixtures, per-record leaf columns); None on every other layout
    mix_mass = mix_w = mix_tab = mix_remap = vcol = None
    leaf_onehot = 0  # pointer walks of one-hot votes: leaves as {class, weight} pairs

    WIDE_G = 4  # tree groups of the wide kernel (mirrors csrc)

    def __init__(self, compiled, device, layout: str = "auto", lds_budget: int = 80 * 1024, splits: int = 0,
                 variant: str = "auto", precision: str = "fp32", nan_mode: str = "auto", max_chunk_trees: int = 0,
                 tree_shard: Optional[Tuple[int, int]] = None, head_depth: int = 0,
                 pointer_schedule: str = "lockstep", node_order: str = "bfs", node_format: str = "wide",
                 pointer_ilp: int = 8, xcd_split: str = "off", pointer_load: str = "auto",
                 hybrid_tail: str = "compact", pointer_leaf: str = "table"):
        """``pointer_leaf`` (lock-step pointer walk): ``"table"`` (a walk ends on a ``~leaf`` code and
        gathers the leaf payload) or ``"inline"`` (leaf payloads of sum ensembles and unit votes sit
        in the parent node's child field: no leaf gather, ``VAR_POINTER_INLINE``).

        ``pointer_load`` (pointer lock-step kernel, features in LDS): ``"clamped"`` (finished walks
        re-load node 0, no branch), ``"masked"`` (their loads are exec-masked off) or ``"uskip"``
        (a walk slot finished in every lane of the wave issues no load at all: wave-uniform branch)
        or ``"peel"`` (the top two levels from wave-uniform scalar loads + a per-lane select),
        ``"ltop"`` (BFS order: levels 0-4 of each lock-step group's trees staged in LDS), or
        ``"auto"`` (default): ltop (BFS) / peel (DFS order) for the 8-walk lock-step kernel with
        table leaves, else clamped. Measured (profiles/r6l, 300 trees x depth 14, 1M rows,
        bit-identical walks): GBDT ltop 2.415 / peel 2.57 / clamped 2.79 ms, RF 3.11 / 3.48 / 3.52.

        ``hybrid_tail`` (hybrid layout): ``"compact"`` (depth-first uint2 tail,
        :func:`~flink_jpmml_amd.runtime.hybrid.pack_hybrid_compact`) or ``"wide"`` (the 16-byte BFS
        pointer tail of :func:`~flink_jpmml_amd.runtime.hybrid.pack_trees`, clamped loads, or
        the wave-uniform skip with ``pointer_load="uskip"``; head depths 2-4). Measured slower than
        the plain pointer walk (profiles/r3ar), kept as a tested option.

        ``xcd_split`` (pointer / hybrid layouts): ``"on"`` splits the forest into 8 tree slices
        scored by workgroups placed on the 8 XCDs (csrc ``tree_block``), so each XCD's 4 MiB L2
        holds one slice instead of the whole forest; ``"off"`` (default): grid.y splits only.
        Measured (profiles/r3q): no gain on a 14 MB depth-14 forest — its L2 hit rate is already
        96 % unsplit; the walk is bound by the vector cache's per-line tag rate (26 distinct lines
        per gather instruction, ~1.3 line accesses per clock per CU), not by L2 capacity.

        ``pointer_schedule`` (pointer layout): ``"lockstep"`` (default: groups of walks run to the
        deepest one; tree-order sums) or ``"refill"`` (each walk slot restarts on the next tree the
        step its walk ends). Measured (profiles/r3j): refill is 2.3-2.6x SLOWER at depth 14 — lanes
        drift onto different trees and every load instruction touches up to 64 distinct lines,
        while lock-step lanes share the lines of the same tree level. ``node_order``: pointer-node
        storage order (``"bfs"``: level by level, siblings adjacent; ``"dfs"``: preorder).
        ``node_format`` (pointer layout): ``"super"``: two tree levels per 16-byte slot
        (:func:`~flink_jpmml_amd.runtime.hybrid.pack_super`, <= 32 features), ``"wide"`` (default) 16-byte nodes, ``"compact"`` 8-byte
        BFS slots with inline leaves (:func:`~flink_jpmml_amd.runtime.hybrid.pack_compact_bfs`;
        features staged in LDS, i.e. at most 64) — measured 1.34x SLOWER (profiles/r3n), kept as
        an option; ``"auto"``: compact whenever it applies. ``pointer_ilp``: walks per lane in
        lock-step (4, 8 or 16; regression sums with features in LDS).

        ``nan_mode`` (wide PERFECT kernel): ``"auto"`` keeps tiles with missing values on the fast
        traversal whenever the ensemble has no null-on-missing trees (default-right nodes read a
        NaN -> +inf second feature plane, :func:`_nan_planes`); ``"off"``: per-node missing test.

        ``tree_shard=(rank, world)``: keep only this rank's contiguous slice of the ensemble and
        emit the RAW weighted leaf sum (the full epilogue is kept in ``full_epi`` and applied after
        the cross-rank ``all_reduce``, :mod:`flink_jpmml_amd.parallel.tree_shard`)."""
        super().__init__(compiled, device)
        if nan_mode not in ("auto", "off"):
            raise ValueError("nan_mode must be 'auto' or 'off'")
        if pointer_ilp not in (2, 4, 6, 8, 16):
            raise ValueError("pointer_ilp must be 2, 4, 6 (LTOP only), 8 or 16")
        self.pointer_ilp = int(pointer_ilp)
        if pointer_schedule not in ("refill", "lockstep"):
            raise ValueError("pointer_schedule must be 'refill' or 'lockstep'")
        self.heads, self.head_depth = None, 0  # hybrid layout only
        self.lds_chunks = self.lds_slices = None  # lds node format only
        self.lds_rows = self.lds_chunk_u4 = self.lds_n_slices = 0
        self.rank_thr, self.rank_cnt, self.rank_stride = None, None, 0  # rank3 node format only
        if pointer_load not in ("auto", "clamped", "masked", "uskip", "peel", "ltop"):
            raise ValueError("pointer_load must be 'auto', 'clamped', 'masked', 'uskip', 'peel' or 'ltop'")
        if pointer_load == "auto":
            pointer_load = (("ltop" if node_order == "bfs" else "peel") if (pointer_ilp == 8 and pointer_leaf == "table")
                            else "clamped")
        if hybrid_tail not in ("compact", "wide"):
            raise ValueError("hybrid_tail must be 'compact' or 'wide'")
        if pointer_leaf not in ("table", "inline"):
            raise ValueError("pointer_leaf must be 'table' or 'inline'")
        self.tail_format = 0
        if xcd_split not in ("on", "off"):
            raise ValueError("xcd_split must be 'on' or 'off'")
        self.xcd_split = 0
        if precision not in ("fp32", "fp8"):
            raise ValueError("tree leaf precision must be fp32 or fp8")
        if layout == "general":
            spec = self._general_spec(compiled)
        else:
            try:
                spec = ensemble_spec(compiled)
            except NotBinaryForm:
                if layout != "auto":
                    raise
                spec, layout = self._general_spec(compiled), "general"
        self.full_epi, self.labels = dict(spec.epi), spec.labels
        if spec.C > 16:
            raise NotLowerable(f"{spec.C} class slots: the tree kernels accumulate at most 16")
        if tree_shard is not None:
            if layout == "general":
                raise NotLowerable("tree sharding needs the binary (perfect / pointer) layouts")
            spec = shard_spec(spec, *tree_shard)
        self.spec = spec
        self.epi_args = dict(spec.epi)
        F = compiled.n_features
        depth = max(1, max(t.depth for t in spec.trees))
        self.depth = depth
        self.n_trees = len(spec.trees)
        if layout == "general":
            if precision == "fp8":
                raise NotLowerable("fp8 leaves need the PERFECT layout")
            from .general_tree import pack_general

            if spec.mode == "slot" and any(b != 0.0 for b in (spec.acc_init or [])):
                raise NotLowerable("K-class chains with intercepts over non-binary trees are host-only")
            spec = to_general(spec)
            self.spec = spec
            self.n_trees = len(spec.trees)

            g = pack_general(spec.trees, spec.weights, spec.P, compiled.schema)
            self.mode, self.tree_w, self.acc_init, self.feat_map = 0, None, None, None
            self.rows_wide, self.n_stage = TB, F
            self.layout, self.variant, self.rec_words, self.chunk_trees = "general", 0, 0, 0
            self.blob_nan, self.chunk_trees_nan = None, 0
            self.P, self.C = spec.P, spec.C
            self.general = 1 if spec.P > 1 else 0
            self.blob = self._t(g["nodes"].reshape(-1))
            self.children = self._t(g["children"])
            self.preds = self._t(g["preds"].reshape(-1))
            self.pool = self._t(g["pool"])
            self.trees_tab = self._t(g["trees"].reshape(-1))
            self.leaves = self._t(g["payload"].reshape(-1))
            mix = g["mix_mass"] is not None
            self.mix_mass = self._t(g["mix_mass"].reshape(-1)) if mix else None
            self.mix_w = self._t(g["mix_w"]) if mix else None
            self.mix_tab = self._t(g["mix_tab"].reshape(-1)) if mix else None
            self.mix_remap = self._t(g["remap"]) if mix else None
            self.vcol = self._t(g["vcol"]) if g["vcol"] is not None else None
            self.roots = None
            self.max_steps = g["max_steps"]
            self.has_dr = False
            self.table = self._t(_label_table(spec.labels)) if spec.labels is not None else None
            self.slots = self._t(np.zeros(self.n_trees, dtype=np.int32)) if self.general else None
            self.splits = 1
            self._partial = None
            return
        self.children = self.preds = self.pool = self.trees_tab = None
        self.max_steps = 0
        self.heads, self.head_depth = None, 0
        NI, NL = (1 << depth) - 1, 1 << depth
        # wide kernel geometry: stage only the columns the trees read (+ columns whose preparation
        # can reject a row); row tiles of 256 / 128 / 64 rows keep the feature planes <= 64 KiB
        stage = self._stage_columns(compiled, spec.trees)
        rows = next((r for r, lim in ((256, 64), (128, 128), (64, 256)) if len(stage) <= lim), None)
        wide_ok = (spec.P == 1 and depth <= 10 and rows is not None and variant != "narrow"
                   and (spec.mode == "sum" or spec.C <= 8))
        if layout == "auto":
            rec_bytes = 4 * (2 * NI + NL * spec.P + (NI + 31) // 32)
            # deeper trees: the POINTER walk (profiles/r3q: 300 trees x depth 14, pointer 3.39 /
            # 2.60 ms vs hybrid-head 4.55 / 3.11 ms for the forest / GBDT)
            layout = "perfect" if depth <= 10 and (wide_ok or F <= 64) and rec_bytes <= 32 * 1024 else "pointer"
        if spec.mode != "sum" and not (layout == "perfect" and wide_ok):
            spec = to_general(spec)  # votes / class slots accumulate in LDS on the narrow kernels
            self.n_trees = len(spec.trees)  # + constant stumps carrying the per-class intercepts
        self.spec = spec
        self.layout = layout
        self.P, self.C = spec.P, spec.C
        self.general = 1 if (spec.P > 1 or (spec.mode == "sum" and spec.slots is not None)) else 0
        self.mode = {"sum": 0, "slot": 1, "class": 2}[spec.mode]
        self.tree_w = self.acc_init = self.feat_map = None
        self.rows_wide, self.n_stage = TB, F
        if self.layout == "perfect":
            if variant == "auto":
                variant = "narrow" if self.general or not wide_ok else "wide"
            self.variant = 1 if variant == "wide" else 0
            if self.variant == 1:
                if not wide_ok:
                    raise NotLowerable("the wide tree kernel needs P = 1 and <= 256 staged columns")
                self.rows_wide, self.n_stage = rows, len(stage)
                stride = rows  # [F][rows] planes: traversal reads hit bank row mod 32 (csrc WideGeom)
                fmap = {f: j for j, f in enumerate(stage)}
                if stage != list(range(F)):
                    self.feat_map = self._t(np.array(stage, dtype=np.int32))
            else:
                if F > 64:
                    raise NotLowerable("the narrow perfect kernel stages at most 64 features")
                stride, fmap = TB, None
            leaf_bits = None
            if spec.mode == "class":
                self.mode = self._vote_mode(spec, rows)
                if self.mode == 3:  # VOTE8: packed u8 counters, the leaf is the increment 1 << 8*class
                    leaf_bits = "vote8"
                elif spec.tree_w is not None and any(w != 1.0 for w in spec.tree_w):
                    self.tree_w = self._t(np.asarray(spec.tree_w, np.float32))
            if spec.mode == "slot":
                if spec.acc_init is not None and any(b != 0.0 for b in spec.acc_init):
                    self.acc_init = self._t(np.asarray(spec.acc_init, np.float32))
            blob, rec, has_dr = _perfect_pack(spec.trees, spec.weights, spec.P, depth, stride=stride, fmap=fmap,
                                              leaf_bits=leaf_bits)
            nan_flags = 0
            blob_nan = None
            Fs = self.n_stage
            if self.variant == 1 and nan_mode == "auto" and not any(t.null_missing for t in spec.trees):
                if not has_dr:
                    nan_flags = VAR_NAN_FAST
                elif precision != "fp8" or (2 * Fs - 1) * stride * 4 < (1 << 16):  # fp8 metas: 16-bit offsets
                    blob_nan = _nan_planes(blob, depth, Fs, stride)
                    nan_flags = VAR_NAN_FAST | VAR_NAN_PLANES
            if self.variant == 1 and self.mode == 3 and precision != "fp8" and depth >= 2 \
                    and (Fs * 2 if blob_nan is not None else Fs) * stride * 4 <= (1 << 16):
                # VOTE8 forest: class codes in the last-level metas (no leaf array, no leaf read)
                blob, rec = _vote_codes_pack(blob, depth)
                if blob_nan is not None:
                    blob_nan, _ = _vote_codes_pack(blob_nan, depth)
                self.variant = 2
            if precision == "fp8":
                # e4m3 leaves in the last-level metas, global scale folded into the epilogue
                if self.general or self.variant != 1 or spec.mode != "sum":
                    raise NotLowerable("fp8 leaves need the single-accumulator wide kernel (P = 1)")
                if (Fs - 1) * stride * 4 >= (1 << 16):
                    raise NotLowerable("fp8 leaf pairs need feature offsets below 64 KiB")
                blob, rec, scale = _leaf8_pack(blob, depth)
                if blob_nan is not None:
                    blob_nan, _, _ = _leaf8_pack(blob_nan, depth, scale)
                self.epi_args["a"] = self.epi_args.get("a", 1.0) * scale
                self.variant = 2
            self.variant |= nan_flags
            self.rec_words = rec
            wide = self.variant & 3 in (1, 2)
            dyn = False
            if wide:
                # one 1024-thread workgroup per row tile: [G][rows] partials + feature plane(s) + two
                # chunk buffers; tiles with missing values use the NaN blob with two planes
                G = 1024 // self.rows_wide
                plane = Fs * stride * 4
                dyn = self.mode == 0 and self.rows_wide == 256  # MODE_SUM batch slots (csrc DYN / NPART)
                npart = DYN_SLOTS if dyn else G
                fixed = plane + (self.rows_wide + 4 + 8) * 4 + npart * self.rows_wide * 4
                per_chunk = min((156 * 1024 - fixed) // 2, 64 * 1024)
            else:
                plane = F * TB * 4
                fixed = plane + (TB + 4) * 4 + (self.C * TB * 4 if self.general else 0)
                budget = max(lds_budget - fixed, 2 * rec * 4)  # two chunk buffers (double buffering)
                per_chunk = min(budget // 2, 32 * 1024)  # register prefetch holds <= 32 KiB per chunk
            if rec * 4 > per_chunk:
                raise NotLowerable(f"depth-{depth} tree record ({rec * 4} B) exceeds the chunk buffer")
            cap = DYN_B * DYN_SLOTS if wide and dyn else 0  # dynamic batches: one slot per batch
            self.chunk_trees = self._chunk(per_chunk // (rec * 4), wide, max_chunk_trees, cap)
            self.blob_nan, self.chunk_trees_nan = None, 0
            if blob_nan is not None:
                per_nan = min((156 * 1024 - fixed - plane) // 2, 64 * 1024)
                if rec * 4 <= per_nan:
                    self.chunk_trees_nan = self._chunk(per_nan // (rec * 4), wide, max_chunk_trees, cap)
                    self.blob_nan = self._t(blob_nan.reshape(-1).view(np.int32))
                else:
                    self.variant &= ~(VAR_NAN_FAST | VAR_NAN_PLANES)
            self.blob = self._t(blob.reshape(-1).view(np.int32))
            self.roots = self.leaves = None
        else:
            if precision == "fp8":
                raise NotLowerable("fp8 leaves need the PERFECT layout")
            from .hybrid import head_words, pack_compact_bfs, pack_hybrid_compact, pack_super, pack_trees

            feat_lds = F <= 64
            H = 0
            heads = None
            if self.layout == "hybrid":
                # PERFECT head of the top H levels in LDS + COMPACT depth-first tail from L2
                # (tree_hybrid.hip); H = 4 measured best at depth 14 (profiles/r3c: larger heads
                # pay more for the per-workgroup head copy and LDS bank conflicts than they save)
                H = head_depth or 4
                if H not in ((2, 3, 4) if hybrid_tail == "wide" else (4, 6, 8, 10)):
                    raise ValueError("head_depth must be 4, 6, 8 or 10 (compact tail) or 2-4 (wide tail)")
                fixed = (F * TB * 4 if feat_lds else 0) + TB * 4 + (self.C * TB * 4 if self.general else 0)
                fit = (lds_budget - fixed) // (head_words(H) * 4)
                if fit < 1:
                    raise NotLowerable("no LDS left for a hybrid head chunk")
                # small chunks: the head buffer must not cost occupancy (the tail walk hides L2 latency
                # with waves; profiles/r3e: 234-tree chunks -> 2 workgroups per CU, 1.5x slower)
                self.chunk_trees = int(min(fit, self.n_trees, max_chunk_trees or 32))
                if hybrid_tail == "wide":
                    heads, nodes, leaves, roots, has_dr = pack_trees(spec.trees, spec.weights, spec.P, H, feat_lds)
                    self.tail_format = 2 if pointer_load == "uskip" else 1
                else:
                    try:
                        heads, nodes, leaves, has_dr = pack_hybrid_compact(spec.trees, spec.weights, spec.P, H, F)
                        roots = np.zeros(self.n_trees, dtype=np.int32)
                        if leaves is None:
                            leaves = np.zeros((1, 1), np.float32)
                    except ValueError:
                        self.layout, H, heads, self.chunk_trees = "pointer", 0, None, 0
            else:
                self.chunk_trees = 0
            compact = superl = rank3 = False
            if node_format == "rank3":
                if heads is not None or not feat_lds or pointer_schedule != "lockstep" or F > 32:
                    raise NotLowerable("rank3 pointer layout needs <= 32 features in LDS and the lock-step walk")
                from .hybrid import pack_rank3

                try:
                    nodes, leaves, roots, rthr, rcnt, has_dr = pack_rank3(spec.trees, spec.weights, spec.P, F)
                except ValueError as e:
                    raise NotLowerable(f"rank3 pointer layout: {e}") from e
                rank3 = True
                self.rank_thr, self.rank_cnt = self._t(rthr.reshape(-1)), self._t(rcnt)
                self.rank_stride = int(rthr.shape[1])
                if leaves is None:
                    leaves = np.zeros((1, 1), np.float32)
            elif node_format == "super":
                if heads is not None or not feat_lds or pointer_schedule != "lockstep" or F > 32:
                    raise NotLowerable("super pointer layout needs <= 32 features in LDS and the lock-step walk")
                try:
                    nodes, leaves, roots, has_dr = pack_super(spec.trees, spec.weights, spec.P)
                    roots = roots.view(np.int32)
                    superl = True
                    if leaves is None:
                        leaves = np.zeros((1, 1), np.float32)
                except ValueError as e:
                    raise NotLowerable(f"super pointer layout: {e}") from e
            elif heads is None and feat_lds and pointer_schedule == "lockstep" and node_format != "wide" \
                    and node_order == "bfs":
                try:
                    nodes, leaves, roots, has_dr = pack_compact_bfs(spec.trees, spec.weights, spec.P)
                    compact = True
                    if leaves is None:
                        leaves = np.zeros((1, 1), np.float32)
                except ValueError:
                    if node_format in ("compact", "lds"):
                        raise NotLowerable(f"{node_format} pointer layout does not apply")
                if compact and node_format == "lds":
                    self._lds_chunks(nodes, roots, F, spec)
            elif node_format == "compact":
                raise NotLowerable("compact pointer layout needs features in LDS, lock-step, bfs")
            inline = False
            if heads is None and not compact and not superl and not rank3:
                # inline leaf payloads on the default lock-step walk (sums, or unit votes) unless
                # asked for the leaf table (pointer_leaf="table")
                inline = (pointer_leaf == "inline" and self.layout == "pointer" and pointer_schedule == "lockstep"
                          and pointer_load in ("clamped", "ltop") and pointer_ilp == 8
                          and ((spec.P == 1 and spec.slots is None) or spec.P > 1))
                _, nodes, leaves, roots, has_dr = pack_trees(spec.trees, spec.weights, spec.P, 0, feat_lds,
                                                             order=node_order, inline_leaves=inline)
            self.blob_nan, self.chunk_trees_nan = None, 0
            self.head_depth = H
            self.rec_words = head_words(H) if H else 0
            # pointer walks: refill schedule (each PILP slot restarts on the next tree as soon as
            # its walk ends) unless pinned to the lock-step kernel's tree-order sums
            self.variant = VAR_POINTER_REFILL if (self.layout == "pointer" and pointer_schedule == "refill") else 0
            if rank3:
                self.variant = VAR_POINTER_RANK3
            elif superl:
                self.variant = VAR_POINTER_SUPER
            elif compact and getattr(self, "lds_chunks", None) is not None:
                self.variant = VAR_POINTER_LDS
            elif compact:
                self.variant = VAR_POINTER_COMPACT
            elif pointer_load == "masked" and self.layout == "pointer" and self.variant == 0 and feat_lds:
                self.variant = VAR_POINTER_MASKED  # finished walks skip their node load (exec mask)
            elif pointer_load == "peel" and self.layout == "pointer" and self.variant == 0 and feat_lds:
                self.variant = VAR_POINTER_PEEL  # top two levels from wave-uniform scalar loads
            elif (pointer_load == "ltop" and self.layout == "pointer" and self.variant == 0 and feat_lds
                  and node_order == "bfs" and pointer_ilp in (6, 8)):
                self.variant = VAR_POINTER_LTOP | (VAR_POINTER_INLINE if inline else 0)  # levels 0-4 from LDS
                # staging reads root + 0 .. 30 of every tree: pad so the last tree's stay in bounds
                nodes = np.concatenate([nodes, np.zeros((POINTER_LTOP_NODES, 4), dtype=nodes.dtype)])
            elif pointer_load == "uskip" and self.layout == "pointer" and self.variant == 0 and feat_lds:
                self.variant = VAR_POINTER_USKIP  # slots finished in the whole wave issue no load
            elif inline and self.variant == 0:
                self.variant = VAR_POINTER_INLINE  # leaf payloads inline: no leaf gather
            self.blob = self._t(nodes.reshape(-1).view(np.int32))
            self.leaf_onehot = 0
            if (self.general and self.P > 1 and leaves.size and self.layout == "pointer"
                    and (self.variant in (0, VAR_POINTER_MASKED, VAR_POINTER_USKIP, VAR_POINTER_PEEL, VAR_POINTER_LTOP))):
                # votes: every leaf row has at most one non-zero payload -> {class, weight} pairs
                # (pointer_walk reads one 8-byte pair and updates one slot instead of P)
                L = np.asarray(leaves, dtype=np.float32).reshape(len(leaves), -1)
                nz = L != 0
                if (nz.sum(axis=1) <= 1).all():
                    cls = np.where(nz.any(axis=1), nz.argmax(axis=1), 0).astype(np.int32)
                    w = L[np.arange(len(L)), cls].astype(np.float32)
                    leaves = np.stack([cls, w.view(np.int32)], axis=1).view(np.float32)
                    self.leaf_onehot = 1
            self.leaves = self._t(leaves.reshape(-1))
            self.roots = self._t(roots)
            self.heads = self._t(heads.reshape(-1).view(np.int32)) if heads is not None else None
            if xcd_split == "on":
                self.xcd_split = XCD_SLICES
        if not (self.variant & 3):
            self.mode = 0  # narrow / pointer kernels: plain sums or LDS slot accumulators
        self.has_dr = has_dr
        self.table = self._t(_label_table(spec.labels)) if spec.labels is not None else None
        if self.general or self.mode == 1:
            sl = spec.slots if spec.slots is not None else [0] * self.n_trees
            self.slots = self._t(np.asarray(sl, dtype=np.int32))
        else:
            self.slots = None
        self.splits = 1 if self.mode else splits
        self._partial = None

    LDS_SLICES = 8  # XCD slices of the LDS-resident walk (one per XCD: tree_lds.hip)

    def _lds_chunks(self, nodes, roots, F: int, spec) -> None:
        """Chunk tables of ``node_format="lds"`` (``tree_lds.hip``): 512-row tiles (256 when the
        feature planes leave too little room), the rest of the 160 KiB LDS one chunk buffer."""
        from .hybrid import pack_lds_chunks

        general = spec.P > 1 or (spec.mode == "sum" and spec.slots is not None)
        CA = spec.C if general else 1
        if general and (spec.C > 8 or spec.P > 8):
            raise NotLowerable("lds pointer layout: at most 8 class slots")
        last = None
        for rows in (512, 256):
            G = 1024 // rows
            head = F * rows * 4 + rows * 4 + G * CA * rows * 4 + 256 * 4  # + the chunk's roots (csrc LROOTS)
            chunk_u4 = min((160 * 1024 - head) // 16, 6 * 1024)  # csrc: LPREF x 1024 uint4 prefetched
            if chunk_u4 < 1024:
                continue
            try:
                chunks, slices = pack_lds_chunks(nodes.shape[0], roots, chunk_u4, self.LDS_SLICES)
            except ValueError as e:
                last = e
                continue
            self.lds_rows, self.lds_chunk_u4 = rows, int(chunk_u4)
            self.lds_chunks = self._t(chunks.reshape(-1))
            self.lds_slices = self._t(slices)
            self.lds_n_slices = int(slices.size - 1)
            return
        raise NotLowerable(f"lds pointer layout: {last or 'no room for a chunk buffer'}")

    def _launch_lds(self, a, n: int, stream) -> None:
        import ctypes

        import torch

        from ..ops._lib import LdsTreeArgs, check, ptr, stream_handle

        S = int(self.lds_n_slices)
        a.partial = None
        if S > 1:
            CA = self.C if self.general else 1
            need = S * (CA + 1) * n
            if self._partial is None or self._partial.numel() < need:
                if self._partial is not None:
                    self.__dict__.setdefault("_retired", []).append(self._partial)
                self._partial = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=self.device)
            a.partial = ptr(self._partial)
        la = LdsTreeArgs()
        la.t = a
        la.chunks, la.slice_chunk = ptr(self.lds_chunks), ptr(self.lds_slices)
        la.n_slices, la.chunk_u4, la.rows = S, int(self.lds_chunk_u4), int(self.lds_rows)
        check(self.lib.pmml_tree_lds_launch(stream_handle(stream), ctypes.byref(la)),
              f"tree kernel (lds, depth {self.depth})")

    @staticmethod
    def _stage_columns(compiled, trees) -> List[int]:
        """Active-field columns the wide kernel stages: every feature a split reads, plus every
        field whose preparation can reject the row (its validity must still be checked)."""
        used = set()
        for t in trees:
            used.update(int(f) for f in t.feature if f >= 0)
        prep, _ = build_field_prep(compiled, compiled.active_fields) if compiled.active_fields else (None, False)
        if prep is not None:
            for j in range(len(compiled.active_fields)):
                if prep[j, 0] & (FP_INVALID_RETURN | FP_ROW_INVALID | FP_INTEGER | FP_CODE_RANGE | FP_HAS_INTERVAL | FP_VALUE_MASK):
                    used.add(j)
        return sorted(used) if used else [0]

    def _vote_mode(self, spec, rows) -> int:
        """MODE_VOTE8 (packed u8 counters, one add per tree) when the vote is unweighted, <= 4
        classes, no leaf lacks a class and no thread's counter can pass 255; else MODE_CLASS."""
        G = 1024 // (rows or 256)
        unweighted = spec.tree_w is None or all(w == 1.0 for w in spec.tree_w)
        no_nan = all(not np.isnan(t.leaf_value[t.feature < 0]).any() for t in spec.trees)
        if unweighted and spec.C <= 4 and no_nan and -(-len(spec.trees) // G) <= 255:
            return 3
        return 2

    def _chunk(self, fit: int, wide: bool, cap: int, slot_cap: int = 0) -> int:
        """Trees per LDS chunk. Wide kernel: whole ILP batches per tree group (G groups x 8-wide
        walks) — every group gets the same count (no barrier imbalance) and no latency-bound short
        tail batches (measured: 64 > 79 > 57 trees at depth 6). MODE_SUM claims 8-tree batches
        dynamically: whole batches, at most ``slot_cap`` trees (one LDS slot per batch)."""
        c = int(max(1, min(self.n_trees, fit)))
        if slot_cap:
            c = min(c, slot_cap)
        G = 1024 // getattr(self, "rows_wide", 256)
        if wide and c < self.n_trees:
            q = DYN_B if slot_cap else (8 * G if c >= 16 * G else 2 * G)
            c = max(q, c // q * q) if c >= q else c
        return min(c, cap) if cap > 0 else c

    @staticmethod
    def _general_spec(compiled) -> "EnsembleSpec":
        from .general_tree import lower_general_tree

        try:
            spec = ensemble_spec(compiled, lower=lower_general_tree)
            if spec.mode == "slot" and any(b != 0.0 for b in (spec.acc_init or [])):
                raise NotLowerable("K-class chains with intercepts over non-binary trees are host-only")
            # sibling-mixture trees (weightedConfidence / aggregateNodes) add their normalised
            # mixture (or its argmax vote) themselves: they need their segment weight, vote mode
            # and category slots before to_general folds them into the leaf payloads
            for i, t in enumerate(spec.trees):
                if getattr(t, "mix_mass", None) is None:
                    continue
                if spec.mode == "class":
                    t.mix_vote, t.mix_weight = True, float((spec.tree_w or [1.0] * len(spec.trees))[i])
                elif spec.mode == "sum" and spec.P > 1 and spec.slots is None:
                    t.mix_vote, t.mix_weight = False, float(spec.weights[i])
                else:
                    raise NotLowerable("sibling mixture trees inside this ensemble form are host-only")
                cats = list(spec.labels or [])
                tc = list(t.ev.categories)
                if any(c not in cats for c in tc):
                    raise NotLowerable("tree category outside the ensemble's classes")
                t.mix_remap = np.array([cats.index(c) for c in tc], dtype=np.int32)
            return to_general(spec)  # the predicate VM accumulates P = C payloads in LDS
        except NotBinary as e:  # pragma: no cover - the general lowering never raises NotBinary
            raise NotLowerable(str(e)) from e

    def _post_state(self) -> None:
        self._partial = None
        self._args = {}
        self._args_buf = {}

    def _args_template(self, with_probs: bool):
        """Per-plan cached argument struct (only row pointers change per launch: keeps the host
        cost of a launch in the few-µs range)."""
        import ctypes

        from ..ops._lib import TreeArgs, ptr

        cache = self.__dict__.setdefault("_args", {})
        a = cache.get(with_probs)
        if a is None:
            a = TreeArgs()
            a.prep = ptr(self.prep)
            a.blob, a.roots, a.leaves, a.tree_slot = ptr(self.blob), ptr(self.roots), ptr(self.leaves), ptr(self.slots)
            a.n_trees, a.rec_words, a.chunk_trees, a.P = self.n_trees, self.rec_words, self.chunk_trees, self.P
            a.C, a.general, a.variant = self.C, self.general, self.variant
            a.blob_nan, a.chunk_trees_nan = ptr(getattr(self, "blob_nan", None)), getattr(self, "chunk_trees_nan", 0)
            a.tree_w, a.acc_init = ptr(getattr(self, "tree_w", None)), ptr(getattr(self, "acc_init", None))
            a.feat_map = ptr(getattr(self, "feat_map", None))
            a.rows_wide, a.mode = getattr(self, "rows_wide", TB), getattr(self, "mode", 0)
            a.n_stage = getattr(self, "n_stage", self.n_features)
            a.pilp = getattr(self, "pointer_ilp", 8)
            a.prof = ptr(getattr(self, "prof", None))  # kbench --tree-prof phase timers (nullable)
            a.rank_thr, a.rank_cnt = ptr(getattr(self, "rank_thr", None)), ptr(getattr(self, "rank_cnt", None))
            a.rank_stride = int(getattr(self, "rank_stride", 0) or 0)
            a.leaf_onehot = int(getattr(self, "leaf_onehot", 0) or 0)
            a.epi = _epilogue(table=self.table, write_probs=with_probs, **self.epi_args)
            cache[with_probs] = a
        # one mutable copy per thread, reused across launches: the C launcher copies the struct
        # before returning, and every per-launch field is rewritten by launch()
        bufs = self.__dict__.setdefault("_args_buf", {})
        key = (threading.get_ident(), with_probs)
        b = bufs.get(key)
        if b is None:
            if len(bufs) > 64:  # threads come and go (loader / job threads): bounded
                bufs.clear()
            b = bufs[key] = TreeArgs()
        ctypes.pointer(b)[0] = a
        return b

    def _auto_splits(self, n_rows: int) -> int:
        if self.splits:
            return self.splits
        blocks = (n_rows + TB - 1) // TB
        if getattr(self, "xcd_split", 0) and self.n_trees >= 2 * XCD_SLICES:
            return XCD_SLICES
        if self.layout == "perfect" and self.variant & 3 and self.n_trees >= 64:
            # wide kernel (one 1024-thread workgroup per 256-row tile): about one workgroup per CU
            # and at most 16 tree slices — measured best for 256-64K rows (profiles/r3y/splits.jsonl:
            # 4096 rows 16.9 us at 16 slices vs 25.4 / 42.6 us at 32 / 62, 64K rows 83 us unsplit)
            return int(max(1, min(16, 256 // max(1, blocks), self.n_trees // 8)))
        target = 512  # ~2 workgroups per CU on 256 CUs
        if blocks >= target or self.n_trees < 64:
            return 1
        return int(max(1, min(self.n_trees // 16, target // max(1, blocks), 64)))

    supports_direct = True  # epilogue can write straight into zero-copy host memory (+ mirror)

    def launch(self, X, score, valid, stream=None, probs=None, row_valid=None, splits: Optional[int] = None,
               score2=None, valid2=None) -> None:
        import ctypes

        import torch

        from ..ops._lib import TreeArgs, check, ptr, stream_handle

        n = X.shape[0]
        if X.shape[1] == 0:
            # feature-less trees (single leaves, e.g. a chain segment with an empty MiningSchema):
            # the kernels still stage one column, so hand them a real one instead of a 0-wide
            # tensor whose data pointer owns no bytes
            X = torch.zeros((n, 1), dtype=torch.float32, device=X.device)
        if self.layout == "general":
            self._launch_general(X, score, valid, stream, probs, row_valid, score2, valid2)
            return
        s = splits if splits is not None else self._auto_splits(n)
        a = self._args_template(probs is not None)
        a.X = X.data_ptr()
        a.n_rows, a.n_feat, a.ldx = n, X.shape[1], X.stride(0)
        a.row_valid_in = ptr(row_valid)
        a.score, a.valid, a.probs = _addr(score), _addr(valid), ptr(probs)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.partial = None
        a.xcd_split = 1 if getattr(self, "xcd_split", 0) and s > 1 else 0
        if s > 1:
            need = s * (self.C + 1) * n
            if self._partial is None or self._partial.numel() < need:
                if self._partial is not None:
                    # an in-flight kernel on another stream may still use it: never hand it back
                    self.__dict__.setdefault("_retired", []).append(self._partial)
                self._partial = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=self.device)
            a.partial = ptr(self._partial)
        if self.variant & VAR_POINTER_LDS:
            self._launch_lds(a, n, stream)
            return
        if self.layout == "hybrid":
            from ..ops._lib import HybridArgs

            h = HybridArgs()
            h.t = a
            h.heads, h.head_words = ptr(self.heads), int(self.rec_words)
            h.tail_format = int(getattr(self, "tail_format", 0))
            rc = self.lib.pmml_tree_hybrid_launch(stream_handle(stream), ctypes.byref(h), int(self.head_depth), s)
            check(rc, f"tree kernel (hybrid, head {self.head_depth}, depth {self.depth})")
            return
        rc = self.lib.pmml_tree_launch(stream_handle(stream), ctypes.byref(a), 0 if self.layout == "perfect" else 1,
                                       self.depth, 1 if self.has_dr else 0, s)
        check(rc, f"tree kernel ({self.layout}, depth {self.depth})")


    def row_launcher(self, X, score, valid):
        """A launch of this plan over FIXED buffers (``StreamingScorer.score_row``'s persistent
        row): the argument block (and the split partials) are built once, and each call only hands
        the block to the C launcher -- the per-call Python of :meth:`launch` was a third of a
        per-record predict. None for the layouts with launchers of their own."""
        if self.layout not in ("perfect", "pointer") or self.variant & VAR_POINTER_LDS or X.shape[1] == 0:
            return None
        import ctypes

        import torch

        from ..ops._lib import TreeArgs, check, stream_handle

        n = X.shape[0]
        s = self._auto_splits(n)
        a = TreeArgs()
        ctypes.memmove(ctypes.byref(a), ctypes.byref(self._args_template(False)), ctypes.sizeof(TreeArgs))
        a.X = X.data_ptr()
        a.n_rows, a.n_feat, a.ldx = n, X.shape[1], X.stride(0)
        a.row_valid_in = None
        a.score, a.valid, a.probs = _addr(score), _addr(valid), None
        a.epi.score2, a.epi.valid2 = None, None
        a.partial = None
        a.xcd_split = 1 if getattr(self, "xcd_split", 0) and s > 1 else 0
        partial = None
        if s > 1:
            partial = torch.empty(max(s * (self.C + 1) * n, 1), dtype=torch.float32, device=self.device)
            a.partial = partial.data_ptr()
        lib, layout = self.lib, 0 if self.layout == "perfect" else 1
        depth, dr = self.depth, 1 if self.has_dr else 0

        def run(stream) -> None:
            check(lib.pmml_tree_launch(stream_handle(stream), ctypes.byref(a), layout, depth, dr, s),
                  f"tree kernel ({self.layout}, depth {depth}, row)")

        run.keep = (a, partial, X)  # the block and the buffers it points at live as long as run
        return run

    def batch_launch_args(self, x_ptr: int, n: int, n_feat: int, ldx: int, score_ptr: int, valid_ptr: int):
        """``(TreeArgs, (layout, depth, has_dr, splits))`` of one launch over rows at ``x_ptr``,
        for ``pmml_tree_launch_many`` (several models' launches from one host call), or ``None``
        when this plan launches otherwise (hybrid / general layouts go through :meth:`launch`)."""
        import torch

        from ..ops._lib import TreeArgs, ptr

        if self.layout not in ("perfect", "pointer") or n <= 0 or self.variant & VAR_POINTER_LDS:
            return None
        s = self._auto_splits(n)
        a = TreeArgs.from_buffer_copy(self._args_template(False))
        a.X, a.n_rows, a.n_feat, a.ldx = x_ptr, n, n_feat, ldx
        a.row_valid_in = None
        a.score, a.valid, a.probs = score_ptr, valid_ptr, None
        a.epi.score2, a.epi.valid2 = None, None
        a.partial = None
        a.xcd_split = 1 if getattr(self, "xcd_split", 0) and s > 1 else 0
        if s > 1:
            need = s * (self.C + 1) * n
            if self._partial is None or self._partial.numel() < need:
                if self._partial is not None:
                    self.__dict__.setdefault("_retired", []).append(self._partial)
                self._partial = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=self.device)
            a.partial = ptr(self._partial)
        return a, (0 if self.layout == "perfect" else 1, int(self.depth), 1 if self.has_dr else 0, int(s))

    def grouped_args(self, n_feat: int):
        """``(TreeArgs, depth, key, tile_rows)`` of this plan as one entry of a grouped mixed-model
        launch (``pmml_tree_launch_grouped``: one wide-kernel launch over many models' rows,
        ``runtime/grouped.py``), or ``None`` when it does not score with the wide perfect kernel.
        Entries with equal ``key`` share one launch; the row fields are set on the device."""
        from ..ops._lib import TreeArgs

        if self.layout != "perfect" or not (self.variant & 3) or self.P != 1 or \
                getattr(self, "n_stage", self.n_features) > n_feat:
            return None
        a = TreeArgs.from_buffer_copy(self._args_template(False))
        a.X, a.n_rows, a.n_feat, a.ldx = None, 0, n_feat, n_feat
        a.row_valid_in, a.score, a.valid, a.probs, a.partial, a.prof = None, None, None, None, None, None
        a.epi.score2, a.epi.valid2 = None, None
        a.xcd_split, a.trees_per_split = 0, self.n_trees
        rows = int(a.rows_wide)
        return a, int(self.depth), (int(self.depth), int(self.variant & 3), rows, int(a.mode)), rows

    def _launch_general(self, X, score, valid, stream, probs, row_valid, score2, valid2) -> None:
        import ctypes

        from ..ops._lib import GenTreeArgs, check, ptr, stream_handle

        g = GenTreeArgs()
        g.t = self._args_template(probs is not None)
        g.t.X = X.data_ptr()
        g.t.n_rows, g.t.n_feat, g.t.ldx = X.shape[0], X.shape[1], X.stride(0)
        g.t.row_valid_in = ptr(row_valid)
        g.t.score, g.t.valid, g.t.probs = _addr(score), _addr(valid), ptr(probs)
        g.t.epi.score2, g.t.epi.valid2 = _addr(score2), _addr(valid2)
        g.t.partial = None
        g.nodes, g.children, g.preds = ptr(self.blob), ptr(self.children), ptr(self.preds)
        g.pool, g.trees, g.max_steps = ptr(self.pool), ptr(self.trees_tab), int(self.max_steps)
        g.mix_mass, g.mix_w = ptr(getattr(self, "mix_mass", None)), ptr(getattr(self, "mix_w", None))
        g.mix_tab, g.remap = ptr(getattr(self, "mix_tab", None)), ptr(getattr(self, "mix_remap", None))
        g.vcol = ptr(getattr(self, "vcol", None))
        check(self.lib.pmml_tree_general_launch(stream_handle(stream), ctypes.byref(g)), "general tree kernel")


# --------------------------------------------------------------------------- dispatch


def _segmented_plan(compiled, device, fused_error: Exception, opts: dict) -> DevicePlan:
    """A MiningModel the fused ensemble kernels refuse: per-segment plans + device predicates
    (runtime/segmented.py), behind a prepare-only derive pass when the inputs need MiningField
    treatment (segment plans and predicates read prepared columns, as the oracle's do)."""
    from .segmented import ChainPlan, SegmentedPlan, segmentable

    ev = compiled.evaluator
    if getattr(ev, "method", None) == "modelChain":  # general chains: segment outputs feed later segments
        try:
            return _with_prepared_inputs(compiled, device, lambda c: ChainPlan(c, device, **opts), opts)
        except NotLowerable as e:
            raise NotLowerable(f"{fused_error}; modelChain: {e}") from e
    why = segmentable(compiled.evaluator, compiled)
    if why:
        raise NotLowerable(f"{fused_error}; segmentation: {why}") from fused_error
    return _with_prepared_inputs(compiled, device, lambda c: SegmentedPlan(c, device, **opts), opts)


def _with_prepared_inputs(compiled, device, build, opts: dict) -> DevicePlan:
    """``build(compiled)`` for a plan class that reads prepared inputs; when the model's MiningField
    treatment is not the identity, a prepare-only derive pass runs first and the plan is built
    by compile_plan on its (prepared) view."""
    if not getattr(compiled, "prepared_inputs", False):
        _, any_prep = build_field_prep(compiled, compiled.active_fields) if compiled.active_fields \
            else (None, False)
        if any_prep:
            from .derive import DerivedPlan, build_program_layout

            layout = build_program_layout(compiled, {}, list(compiled.active_fields))
            return DerivedPlan(compiled, device, layout, **opts)
    return build(compiled)


def compile_plan(compiled, device, **opts) -> DevicePlan:
    """Pick and build the device plan for a compiled model; raises :class:`NotLowerable` when the
    model needs the host oracle."""
    ev = compiled.evaluator
    if not compiled.target_fields:
        raise NotLowerable("model has no target field (every record scores EmptyScore)")
    if not getattr(compiled, "fields_resolved", False):
        from .design import design_layout, needs_design

        if needs_design(ev):  # categorical predictors / terms / GLM -> design columns + dense GEMV
            from .derive import DerivedPlan

            layout, _ = design_layout(compiled)
            return DerivedPlan(compiled, device, layout, **opts)
        # derived fields: pure casts alias their input column (tree kernels), anything else runs
        # as a derive-kernel pass in front of the model kernel (runtime/derive.py)
        from .derive import DerivedPlan, FieldView, plan_field_layout

        is_tree = isinstance(ev, (TreeEvaluator, MiningEvaluator))
        layout = plan_field_layout(compiled, allow_alias=is_tree, allow_fold=is_tree)
        if layout.folds:  # monotone derived fields folded into the split thresholds (derive.py)
            try:
                prec = "fp8" if opts.get("precision") == "fp8" else "fp32"
                return TreePlan(FieldView(compiled, layout, prepared=False), device, precision=prec,
                                **{k: v for k, v in opts.items() if k != "precision"})
            except NotLowerable:
                layout = plan_field_layout(compiled, allow_alias=True, allow_fold=False)
        if layout.program is not None:
            return DerivedPlan(compiled, device, layout, **opts)
        compiled = FieldView(compiled, layout, prepared=False)
    # ``precision`` is a policy (fp32 | bf16 | fp8, see config.ScoringConfig): trees take fp8 leaves
    # only, neural networks take bf16 (also under fp8), every other family stays fp32
    policy = opts.pop("precision", "fp32")
    if policy not in ("fp32", "bf16", "fp8"):
        raise ValueError(f"precision must be fp32, bf16 or fp8, got {policy!r}")
    if isinstance(ev, ClusteringEvaluator):
        if getattr(ev, "knn", None) is not None and (min(ev.k, len(ev.targets)) > 1 or ev.target is not None):
            return KnnPlan(compiled, device, **opts)
        return ClusterPlan(compiled, device, **opts)
    if isinstance(ev, (TreeEvaluator, MiningEvaluator)):
        try:
            return TreePlan(compiled, device, precision="fp8" if policy == "fp8" else "fp32", **opts)
        except NotLowerable as e:
            if not isinstance(ev, MiningEvaluator):
                raise
            return _segmented_plan(compiled, device, e, dict(opts, precision=policy))
    if isinstance(ev, RegressionEvaluator):
        return LinearPlan(compiled, device)
    from ..models.regression import GeneralRegressionEvaluator

    if isinstance(ev, GeneralRegressionEvaluator):
        raise NotLowerable("GeneralRegressionModel lowers through design columns (runtime/design.py)")
    from ..models.neural import NeuralEvaluator
    from ..models.svm import SvmEvaluator

    if isinstance(ev, NeuralEvaluator):
        from .nn_plans import GemmMlpPlan, MlpPlan, WideMlpPlan

        prec = "fp32" if policy == "fp32" else "bf16"
        impl = opts.pop("mlp_impl", "auto")  # auto | fused | wide | gemm
        if impl not in ("auto", "fused", "wide", "gemm"):
            raise ValueError("mlp_impl must be auto, fused, wide or gemm")

        def build(c):
            if impl == "gemm":
                return GemmMlpPlan(c, device, precision=prec)
            if impl == "wide":
                return WideMlpPlan(c, device, precision=prec)
            try:
                return MlpPlan(c, device, precision=prec, **opts)
            except NotLowerable as e:
                if "fused kernel" not in str(e) or impl == "fused":
                    raise
                try:  # wide layers: one fused MFMA GEMM launch per layer (ops/csrc/gemm.hip), bf16 or fp32
                    return WideMlpPlan(c, device, precision=prec)
                except NotLowerable:  # > 32 outputs or > 16384 inputs: library GEMMs
                    return GemmMlpPlan(c, device, precision=prec)

        # the network kernels read the raw input columns (NormContinuous / mapMissingTo fused into
        # their input stage): a MiningField / DataField treatment that is not the identity
        # (missing replacement, validity intervals, outliers, invalid treatment) runs as a
        # prepare-only derive pass first — the kernels never see unprepared values
        return _with_prepared_inputs(compiled, device, build, dict(opts, precision=policy, mlp_impl=impl))
    if isinstance(ev, SvmEvaluator):
        from .nn_plans import SvmGemmPlan, SvmPlan, SvmWidePlan

        impl = opts.pop("svm_impl", "auto")  # auto | fused | wide | gemm
        if impl not in ("auto", "fused", "wide", "gemm"):
            raise ValueError("svm_impl must be auto, fused, wide or gemm")
        if impl in ("auto", "fused"):
            try:
                return SvmPlan(compiled, device)
            except NotLowerable:
                if impl == "fused":
                    raise
        if impl in ("auto", "wide"):
            try:  # many machines / classes / fields: the two-GEMM fused MFMA kernel
                return SvmWidePlan(compiled, device)
            except NotLowerable:
                if impl == "wide":
                    raise
        return _with_prepared_inputs(compiled, device, lambda c: SvmGemmPlan(c, device),
                                     dict(opts, svm_impl="gemm"))
    raise NotLowerable(f"no device plan for {type(ev).__name__}")
