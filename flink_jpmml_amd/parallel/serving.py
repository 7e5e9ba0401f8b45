"""Dynamic multi-model serving across GPU ranks (one process per GPU).

The reference's dynamic operator (`S/api/functions/EvaluationCoFunction.scala`) runs once per
Flink subtask: every subtask receives the broadcast control stream (`S/package.scala:65`) and
loads every model itself from the distributed file system into an unbounded per-subtask cache
(`EvaluationCoFunction.scala:66-67`). Here the control plane is replicated the same way, and the
model plane has two placements:

* ``placement="replicate"`` (the reference's behaviour, data parallel): on ``Add`` rank 0 reads +
  parses + lowers the PMML **once** and replicates the compiled device tensors over RCCL
  (:func:`broadcast_plan`, F2) — eagerly, so the first event on any rank never pays a parse.
  Events are scored where they arrive (F3) and :meth:`gather` collects the scored shards (F5).
* ``placement="sharded"`` (the expert-parallel analogue for many-model serving): every
  model lives on ONE owner rank (``crc32(model id) % world``), so N GPUs hold N× the models of one
  (288 GB HBM3E each). :meth:`score_routed` routes each event to its model's owner with one
  variable-size ``all_to_all`` (xGMI point-to-point: each pair of GPUs exchanges only its own
  rows), the owner scores its rows per model on its device pipeline, and a second ``all_to_all``
  returns the scores to the rank the events arrived on, in arrival order.

Metadata semantics are exactly the single-process ones (:func:`metadata_manager`), so a
duplicate Add is ignored on every rank and Del evicts everywhere. Scoring goes through
:func:`~flink_jpmml_amd.runtime.engine.make_scorer`: a model the device cannot run follows the
``ScoringConfig.fallback`` policy (``warn`` / ``host`` / ``error``) and is counted — never a silent
oracle fallback; a model evicted from the LRU cache is re-lowered locally (collective-free) under
the same policy.
"""

from __future__ import annotations

import logging
import zlib
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from ..api.batch import PredictionBatch, RecordBatch
from ..api.managers import metadata_manager
from ..api.reader import ModelReader
from ..config import ScoringConfig, merge_config
from ..domain.control import AddMessage, DelMessage, ServingMessage
from ..domain.model_id import ModelId, ModelInfo
from ..utils.faults import Watchdog, guarded_collective, injector
from ..utils.metrics import METRICS
from ..utils.profiling import prange
from .dist import (DistContext, all_gather_object, all_gather_varlen, all_to_all_varlen, broadcast_control,
                   broadcast_object, broadcast_plan)

logger = logging.getLogger(__name__)

PLACEMENTS = ("replicate", "sharded")


class _Entry:
    __slots__ = ("compiled", "scorer")

    def __init__(self, compiled, scorer):
        self.compiled = compiled
        self.scorer = scorer

    @property
    def plan(self):
        return getattr(self.scorer, "plan", None)


class DistributedServing:
    """``config`` (:class:`~flink_jpmml_amd.config.ScoringConfig`) supplies the device, LRU cache
    capacity, fallback policy, lowering options and the watchdog; the legacy keywords override it."""

    def __init__(self, ctx: DistContext, device=None, cache_capacity: Optional[int] = None,
                 plan_opts: Optional[dict] = None, config: Optional[ScoringConfig] = None,
                 placement: str = "replicate"):
        if placement not in PLACEMENTS:
            raise ValueError(f"placement must be one of {PLACEMENTS}")
        self.config = merge_config(config, device=device, cache_capacity=cache_capacity, plan_opts=plan_opts)
        self.ctx = ctx
        self.device = self.config.device if self.config.device is None else self.config.resolve_device(ctx.local_rank)
        self.placement = placement
        self.metadata: Dict[ModelId, ModelInfo] = {}
        self.models: "OrderedDict[ModelId, _Entry]" = OrderedDict()
        self.cache_capacity = self.config.cache_capacity
        self.plan_opts = self.config.lowering_opts()
        self.batches = 0  # micro-batches scored on this rank (fault-injection clock)
        self._pipeline = None
        self._watchdog = Watchdog(self.config.watchdog_s, name=f"serving-{ctx.rank}").start() \
            if self.config.watchdog_s else None

    # ------------------------------------------------------------------ placement
    def owner(self, model_id: Union[ModelId, str]) -> int:
        """Rank that holds ``model_id`` (every rank under ``placement="replicate"``: this one)."""
        if self.placement == "replicate" or not self.ctx.is_distributed:
            return self.ctx.rank
        return zlib.crc32(str(model_id).encode()) % self.ctx.world_size

    def _kick(self) -> None:
        if self._watchdog is not None:
            self._watchdog.kick()

    def close(self) -> None:
        if self._watchdog is not None:
            self._watchdog.stop()
        for e in self.models.values():
            if hasattr(e.scorer, "drain"):
                e.scorer.drain()

    # ------------------------------------------------------------------ control plane
    def apply_control(self, messages: Optional[Sequence[ServingMessage]] = None) -> List[ServingMessage]:
        """Collective: rank 0 passes its control messages, other ranks pass None. Returns the
        replicated messages (in order) after applying them on every rank."""
        self._kick()
        msgs = guarded_collective(broadcast_control, messages, self.ctx, what="control broadcast")
        errors = []
        for m in msgs:
            if isinstance(m, DelMessage):
                self.models.pop(m.model_id, None)
            before = m.model_id in self.metadata
            self.metadata = metadata_manager(m, self.metadata)
            if isinstance(m, AddMessage) and not before:
                if self.placement == "replicate":
                    self._replicate(m)
                elif self.owner(m.model_id) == self.ctx.rank:
                    try:
                        self._load_local(m.model_id, m.path)
                    except Exception as e:  # noqa: BLE001 - reported to every rank below
                        errors.append(f"{m.model_id}: {type(e).__name__}: {e}")
        if self.placement == "sharded" and self.ctx.is_distributed:
            errors = [x for part in all_gather_object(errors, self.ctx, group=self.ctx.group("ctrl")) for x in part]
        if errors:
            from ..api.exceptions import ModelLoadingException

            raise ModelLoadingException("; ".join(errors))
        return msgs

    def _scorer(self, compiled, plan=None, lower_error=None):
        from ..runtime.engine import DevicePipeline, make_scorer

        if self.device is not None and self._pipeline is None:
            self._pipeline = DevicePipeline(self.device, self.config.micro_batch, self.config.pipeline_depth,
                                            self.config.h2d_streams)
        return make_scorer(compiled, self.device, self.config, pipeline=self._pipeline, plan=plan,
                           lower_error=lower_error)

    def _insert(self, mid: ModelId, e: _Entry) -> None:
        self.models[mid] = e
        self.models.move_to_end(mid)
        while len(self.models) > self.cache_capacity:
            old, ev = self.models.popitem(last=False)
            if hasattr(ev.scorer, "drain"):
                ev.scorer.drain()
            METRICS.inc("serving.cache_evictions")

    def _load_local(self, mid: ModelId, path: str) -> _Entry:
        """Collective-free load on this rank (sharded owners, cache-miss reloads, gloo groups)."""
        from ..runtime.compiled import CompiledPmml

        with prange("serving.load"), METRICS.timer("serving.model_load_ms"):
            compiled = CompiledPmml.from_string(ModelReader(path).build_distributed_path(), source=path)
            e = _Entry(compiled, self._scorer(compiled))
        self._insert(mid, e)
        return e

    def _replicate(self, m: AddMessage) -> None:
        from ..runtime.compiled import CompiledPmml

        text = None
        err = None
        if self.ctx.is_root:
            try:
                text = ModelReader(m.path).build_distributed_path()
            except Exception as e:  # noqa: BLE001 - the leader reports, everybody fails together
                err = f"{type(e).__name__}: {e}"
        text, err = broadcast_object((text, err), self.ctx)
        if err is not None:
            from ..api.exceptions import ModelLoadingException

            raise ModelLoadingException(f"model {m.model_id} at {m.path}: {err}")
        with METRICS.timer("serving.model_load_ms"):
            compiled = CompiledPmml.from_string(text, source=m.path)
            if self.device is not None and compiled.target_fields and \
                    (self.ctx.backend == "nccl" or not self.ctx.is_distributed):
                # parse + lower once on the leader, replicate the device tensors over RCCL
                local, lower_error = None, None
                if self.ctx.is_root:
                    try:
                        local = compiled.plan(self.device, **self.plan_opts)
                    except Exception as e:  # noqa: BLE001 - same outcome on every rank
                        lower_error = f"{type(e).__name__}: {e}"
                lower_error = broadcast_object(lower_error, self.ctx)
                plan = broadcast_plan(local, self.ctx, device=self.device) if lower_error is None else None
                scorer = self._scorer(compiled, plan=plan, lower_error=lower_error)
            else:
                scorer = self._scorer(compiled)
        self._insert(m.model_id, _Entry(compiled, scorer))

    # ------------------------------------------------------------------ data plane
    def _entry(self, mid: ModelId) -> Optional[_Entry]:
        e = self.models.get(mid)
        if e is not None:
            self.models.move_to_end(mid)
            METRICS.inc("serving.cache_hits")
            return e
        if mid in self.metadata and self.owner(mid) == self.ctx.rank:
            METRICS.inc("serving.cache_misses")  # evicted: re-lower locally, same fallback policy
            return self._load_local(mid, self.metadata[mid].path)
        return None

    def score_async(self, model_id: Union[str, ModelId], X) -> PredictionBatch:
        """Score rows on this rank; unknown (or deleted) models give all-EmptyScore rows."""
        self._kick()
        injector().on_batch(self.ctx.rank, self.batches)
        self.batches += 1
        mid = model_id if isinstance(model_id, ModelId) else ModelId.from_identifier(model_id)
        n = len(X)
        if self.placement == "sharded" and self.owner(mid) != self.ctx.rank:
            raise ValueError(f"model {mid} lives on rank {self.owner(mid)}: use score_routed")
        e = self._entry(mid)
        if e is None:
            METRICS.inc("serving.unknown_model_rows", n)
            return PredictionBatch.empty(n)
        batch = X if isinstance(X, RecordBatch) else RecordBatch(np.asarray(X))
        if e.compiled.n_features != batch.n_features:
            return PredictionBatch.empty(n)
        METRICS.inc("serving.rows", n)
        return e.scorer.submit_batch(batch)

    def score(self, model_id: Union[str, ModelId], X) -> Tuple[np.ndarray, np.ndarray]:
        pb = self.score_async(model_id, X).wait()
        return pb.scores, pb.valid

    def gather(self, scores: np.ndarray, valid: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """All-gather variable-length scored shards in rank order (F5)."""
        import torch

        dev = self.ctx.device if self.ctx.backend == "nccl" else torch.device("cpu")
        s = guarded_collective(all_gather_varlen, torch.as_tensor(np.asarray(scores, np.float32), device=dev),
                               self.ctx, what="score all-gather")
        v = guarded_collective(all_gather_varlen, torch.as_tensor(np.asarray(valid, np.uint8), device=dev),
                               self.ctx, what="valid all-gather")
        return s.cpu().numpy(), v.cpu().numpy().astype(bool)

    # ------------------------------------------------------------------ model-sharded routing
    def score_routed(self, model_ids: Union[str, Sequence[str]], X) -> Tuple[np.ndarray, np.ndarray]:
        """Collective (every rank calls it, possibly with zero rows): score each row of ``X`` with
        ``model_ids[i]`` on that model's owner rank and return ``(scores, valid)`` in this rank's
        row order. Under ``placement="replicate"`` this is local :meth:`score` per model."""
        import torch

        X = np.asarray(X)
        n = len(X)
        ids = [model_ids] * n if isinstance(model_ids, str) else list(model_ids)
        if len(ids) != n:
            raise ValueError("model_ids must have one entry per row")
        catalog = sorted(str(k) for k in self.metadata)  # identical on every rank (replicated control)
        code_of = {k: i for i, k in enumerate(catalog)}
        codes = np.full(n, -1, np.int64)
        for i, mid in enumerate(ids):
            key = str(ModelId.from_identifier(mid)) if not isinstance(mid, ModelId) else str(mid)
            codes[i] = code_of.get(key, -1)
        if self.placement == "replicate" or not self.ctx.is_distributed:
            return self._score_codes(catalog, codes, X)
        self._kick()
        world = self.ctx.world_size
        owners = np.array([self.owner(catalog[c]) if c >= 0 else self.ctx.rank for c in codes], np.int64)
        order = np.argsort(owners, kind="stable")
        send_counts = np.bincount(owners, minlength=world).tolist()
        dev = self.ctx.device if self.ctx.backend == "nccl" else torch.device("cpu")
        with prange("serving.route"):
            Xs = torch.as_tensor(np.ascontiguousarray(X[order]), device=dev)
            rX, recv_counts = guarded_collective(all_to_all_varlen, Xs, send_counts, self.ctx, what="event routing")
            rc, _ = guarded_collective(all_to_all_varlen, torch.as_tensor(codes[order], device=dev), send_counts,
                                       self.ctx, what="event routing")
        METRICS.inc("serving.routed_rows", int(n - send_counts[self.ctx.rank]))
        s, v = self._score_codes(catalog, rc.cpu().numpy(), rX.cpu().numpy())
        with prange("serving.return"):
            back_s, _ = guarded_collective(all_to_all_varlen, torch.as_tensor(s, device=dev), recv_counts, self.ctx,
                                           what="score return")
            back_v, _ = guarded_collective(all_to_all_varlen, torch.as_tensor(v.astype(np.uint8), device=dev),
                                           recv_counts, self.ctx, what="score return")
        scores = np.empty(n, np.float64)
        valid = np.empty(n, bool)
        scores[order] = back_s.cpu().numpy()
        valid[order] = back_v.cpu().numpy().astype(bool)
        return scores, valid

    def _score_codes(self, catalog: List[str], codes: np.ndarray, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Score rows grouped by model code on this rank (all groups submitted before any wait)."""
        n = len(codes)
        scores = np.full(n, np.nan)
        valid = np.zeros(n, bool)
        pending = []
        for c in np.unique(codes):
            rows = np.nonzero(codes == c)[0]
            if c < 0:
                METRICS.inc("serving.unknown_model_rows", len(rows))
                continue
            pending.append((rows, self.score_async(catalog[c], X[rows])))
        for rows, pb in pending:
            pb.wait()
            scores[rows] = pb.scores
            valid[rows] = pb.valid
        return scores, valid


__all__ = ["DistributedServing", "PLACEMENTS"]
