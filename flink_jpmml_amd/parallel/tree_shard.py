"""Tree-sharded ensembles: tensor parallelism over the trees of one model (SURVEY §2.7 "TP",
§5.7 "ensemble size scales ... optionally by tree-sharding across GPUs with all-reduce").

The reference only has Flink operator data parallelism (every subtask holds the whole model:
`S/api/functions/EvaluationFunction.scala:43`). For latency-bound serving of very large
ensembles the MI355X form splits the *trees* instead of the records:

* every rank lowers only its contiguous slice of the ensemble (``TreePlan(tree_shard=...)``,
  :func:`flink_jpmml_amd.runtime.plans.shard_spec`) and its kernel writes the RAW weighted leaf
  sum ``Σ w_i·leaf_i`` (plus a per-row valid byte: a null-on-missing tree poisons its rows);
* one ``all_reduce(SUM)`` of the fp32 partial sums (4 B/row) and one ``all_reduce(MIN)`` of the
  valid bytes over RCCL/xGMI combine the shards — a 4096-row batch is 16 KiB, far below one
  link's per-step latency, so the collective costs its launch latency only;
* the model's real epilogue (target affine ``a·z + b``, link, binary-chain threshold and label
  table) is applied after the reduction (:func:`finish_epilogue`), with exactly the semantics of
  ``csrc/epilogue.h::apply_epilogue``.

Supported: single-score ensembles (regression GBDT / forests, the ``modelChain`` binary
calibrator); multi-class ensembles keep data parallelism. On ranks without a GPU (gloo tests)
the partial sums come from :func:`host_partial`, a float64 traversal of the same lowered trees.
"""

from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..models.tree import OP_GE, OP_GT, OP_LE, OP_LT
from ..runtime.plans import (EPI_AFFINE, EPI_LOGISTIC2, NotLowerable, _label_table, apply_target_torch, ensemble_spec,
                             shard_spec)
from .dist import DistContext


def apply_link(link: int, y: torch.Tensor) -> torch.Tensor:
    """Torch twin of ``csrc/common.h::apply_link``."""
    if link == 1:
        return torch.sigmoid(y)
    if link == 2:
        return torch.exp(y)
    if link == 3:
        return 0.5 * torch.erfc(-y * 0.70710678118654752)
    if link == 4:
        return 1.0 - torch.exp(-torch.exp(y))
    if link == 5:
        return torch.exp(-torch.exp(-y))
    if link == 6:
        return 0.5 + torch.atan(y) * 0.31830988618379067
    return y


def finish_epilogue(raw: torch.Tensor, valid: torch.Tensor, epi: dict, labels=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Apply a single-accumulator epilogue (AFFINE / LOGISTIC2) to reduced raw sums.

    Returns ``(score fp32, valid bool)``; invalid rows score NaN (``EmptyScore``)."""
    z = epi.get("a", 1.0) * raw + epi.get("b", 0.0)
    y = apply_link(int(epi.get("link", 0)), z)
    ok = valid.bool()
    if epi["mode"] == EPI_AFFINE:
        s = y
        ok = ok & torch.isfinite(s)
        s, ok = apply_target_torch(s, ok, epi.get("tgt"))
    elif epi["mode"] == EPI_LOGISTIC2:
        label = (y < epi.get("thr", 0.5)).long()  # p0 >= thr -> class 0
        ok = ok & ~torch.isnan(y)
        if labels is not None:
            # the kernel's table: non-numeric labels are NaN -> the row is invalid (EmptyScore)
            tab = torch.as_tensor(_label_table(list(labels)), dtype=raw.dtype, device=raw.device)
            s = tab[label]
        else:
            s = label.to(raw.dtype)
        ok = ok & ~torch.isnan(s)
    else:
        raise ValueError(f"epilogue mode {epi['mode']} is not single-accumulator")
    s = torch.where(ok, s, torch.full_like(s, float("nan")))
    return s.to(torch.float32), ok


def host_partial(spec, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Float64 traversal of a (sharded) spec's pointer-form trees: raw ``Σ w·leaf`` and row validity.

    ``X`` holds the model's input columns already prepared (no MiningField treatment here)."""
    Xf = np.asarray(X, dtype=np.float32).astype(np.float64)
    n = len(Xf)
    rows = np.arange(n)
    acc = np.zeros(n)
    ok = np.ones(n, dtype=bool)
    for t, w in zip(spec.trees, spec.weights):
        node = np.zeros(n, dtype=np.int64)
        saw_missing = np.zeros(n, dtype=bool)
        for _ in range(t.depth + 1):
            f = t.feature[node]
            inner = f >= 0
            if not inner.any():
                break
            x = Xf[rows, np.maximum(f, 0)]
            thr = t.threshold[node]
            op = t.op[node]
            left = np.select([op == OP_LT, op == OP_LE, op == OP_GT, op == OP_GE],
                             [x < thr, x <= thr, x > thr, x >= thr])
            miss = np.isnan(x)
            left = np.where(miss, t.default_left[node], left)
            saw_missing |= inner & miss
            node = np.where(inner, np.where(left, t.left[node], t.right[node]), node)
        acc += w * t.leaf_value[node]
        if t.null_missing:
            ok &= ~saw_missing
    return acc, ok


class TreeShardedScorer:
    """Score full batches with this rank's slice of the trees; combine over ``ctx``'s group.

    Every rank must call :meth:`score` with the same rows (latency mode: the batch is replicated,
    the trees are sharded). ``device=None`` scores on the rank's GPU when it has one, else on the
    host (gloo)."""

    def __init__(self, compiled, ctx: DistContext, device=None, **plan_opts):
        self.ctx = ctx
        self.world, self.rank = max(1, ctx.world_size), ctx.rank
        dev = torch.device(device) if device is not None else ctx.device
        self.device = dev
        self.plan = None
        if dev.type == "cuda":
            from ..runtime.plans import compile_plan

            # compile_plan also handles derived fields (the tree plan then sits behind a derive pass)
            self.plan = compile_plan(compiled, dev, tree_shard=(self.rank, self.world), **plan_opts)
            tp = getattr(self.plan, "inner", self.plan)
            self.epi, self.labels = dict(tp.full_epi), tp.labels
            self.n_trees_local = tp.n_trees
        else:
            if compiled.schema.derived:
                # the host traversal reads raw active-field columns; derived inputs need the derive
                # program only the device plan runs
                raise NotLowerable("host (gloo) tree-shard ranks need a model without derived fields")
            self.compiled = compiled
            full = ensemble_spec(compiled)
            self.epi, self.labels = dict(full.epi), full.labels
            self.spec = shard_spec(full, self.rank, self.world)
            self.n_trees_local = len(self.spec.trees)

    def partial(self, X) -> Tuple[torch.Tensor, torch.Tensor]:
        """This rank's raw partial sums (fp32) and valid bytes (u8) on ``self.device``."""
        if self.plan is not None:
            Xt = torch.as_tensor(X, dtype=torch.float32).to(self.device).contiguous()
            raw, valid = self.plan.alloc_outputs(Xt.shape[0])
            self.plan.launch(Xt, raw, valid)
            return raw, valid
        # MiningField preparation (missing / invalid replacement, outliers) exactly as the device
        # kernels' fused prologue applies it, then the float64 traversal
        P, row_ok = self.compiled.prepare(np.asarray(X, dtype=np.float64))
        acc, ok = host_partial(self.spec, P)
        ok = ok & row_ok
        return torch.from_numpy(acc.astype(np.float32)), torch.from_numpy(ok.astype(np.uint8))

    def score(self, X) -> Tuple[torch.Tensor, torch.Tensor]:
        raw, valid = self.partial(X)
        # rows a shard marked invalid carry NaN partials; zero them so the SUM stays finite and let
        # the MIN over the valid bytes decide
        raw = torch.where(valid.bool(), raw, torch.zeros_like(raw))
        if self.ctx.is_distributed:
            dist.all_reduce(raw, op=dist.ReduceOp.SUM)
            dist.all_reduce(valid, op=dist.ReduceOp.MIN)
        return finish_epilogue(raw, valid, self.epi, self.labels)


def tree_shard_supported(compiled) -> Optional[str]:
    """``None`` when the model can be tree-sharded, else the reason it cannot."""
    try:
        spec = ensemble_spec(compiled)
        shard_spec(spec, 0, 1)
    except Exception as e:  # noqa: BLE001
        return str(e)
    return None
