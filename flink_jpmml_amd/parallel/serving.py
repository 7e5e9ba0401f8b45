"""Data-parallel dynamic multi-model serving across GPU ranks (one process per GPU).

The reference's dynamic operator (`S/api/functions/EvaluationCoFunction.scala`) runs once per
Flink subtask: every subtask receives the broadcast control stream (`S/package.scala:65`) and
loads every model itself from the distributed file system. Here:

* rank 0 is the control-plane leader: it ingests Add/Del messages and replicates them
  (:func:`broadcast_control`, F1);
* on ``Add`` rank 0 reads + parses + lowers the PMML **once** and replicates the compiled device
  tensors over RCCL (:func:`broadcast_plan`, F2) — eagerly, so the first event on any rank never
  pays a parse; on a host-only rank group (``gloo``) the PMML text is replicated instead;
* events are scored where they arrive (host-side sharding, F3); :meth:`gather` collects the
  scored shards (F5).

Metadata semantics are exactly the single-process ones (:func:`metadata_manager`), so a
duplicate Add is ignored on every rank and Del evicts everywhere.
"""

from __future__ import annotations

import logging
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..api.managers import metadata_manager
from ..api.reader import ModelReader
from ..domain.control import AddMessage, DelMessage, ServingMessage
from ..domain.model_id import ModelId, ModelInfo
from ..utils.faults import guarded_collective, injector
from .dist import DistContext, all_gather_varlen, broadcast_control, broadcast_object, broadcast_plan

logger = logging.getLogger(__name__)


class _Entry:
    __slots__ = ("compiled", "plan")

    def __init__(self, compiled, plan):
        self.compiled = compiled
        self.plan = plan


class DistributedServing:
    def __init__(self, ctx: DistContext, device=None, cache_capacity: int = 64, plan_opts: Optional[dict] = None):
        self.ctx = ctx
        self.device = device
        self.metadata: Dict[ModelId, ModelInfo] = {}
        self.models: "OrderedDict[ModelId, _Entry]" = OrderedDict()
        self.cache_capacity = cache_capacity
        self.plan_opts = plan_opts or {}
        self.batches = 0  # micro-batches scored on this rank (fault-injection clock)

    # ------------------------------------------------------------------ control plane
    def apply_control(self, messages: Optional[Sequence[ServingMessage]] = None) -> List[ServingMessage]:
        """Collective: rank 0 passes its control messages, other ranks pass None. Returns the
        replicated messages (in order) after applying them on every rank."""
        msgs = guarded_collective(broadcast_control, messages, self.ctx, what="control broadcast")
        for m in msgs:
            if isinstance(m, DelMessage):
                self.models.pop(m.model_id, None)
            before = m.model_id in self.metadata
            self.metadata = metadata_manager(m, self.metadata)
            if isinstance(m, AddMessage) and not before:
                self._replicate(m)
        return msgs

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
        compiled = CompiledPmml.from_string(text, source=m.path)
        plan = None
        if self.device is not None:
            on_gpu = self.ctx.backend == "nccl" or not self.ctx.is_distributed
            if on_gpu:
                local = None
                ok = True
                if self.ctx.is_root:
                    try:
                        local = compiled.plan(self.device, **self.plan_opts)
                    except Exception as e:  # noqa: BLE001
                        ok = False
                        logger.warning("model %s not lowerable (%s): host scoring", m.model_id, e)
                ok = broadcast_object(ok, self.ctx)
                if ok:
                    plan = broadcast_plan(local, self.ctx, device=self.device)
        self.models[m.model_id] = _Entry(compiled, plan)
        self.models.move_to_end(m.model_id)
        while len(self.models) > self.cache_capacity:
            self.models.popitem(last=False)

    # ------------------------------------------------------------------ data plane
    def score(self, model_id: str, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Score this rank's shard for ``model_id``; unknown models give all-invalid rows."""
        injector().on_batch(self.ctx.rank, self.batches)
        self.batches += 1
        mid = ModelId.from_identifier(model_id)
        e = self.models.get(mid)
        if e is None:
            if mid in self.metadata:  # evicted from the cache: reload (collective-free path)
                from ..runtime.compiled import CompiledPmml

                e = _Entry(CompiledPmml.load(self.metadata[mid].path), None)
                self.models[mid] = e
            else:
                n = len(X)
                return np.full(n, np.nan), np.zeros(n, dtype=bool)
        if e.plan is not None:
            s, v = e.plan.score(X)
            return s.cpu().numpy(), v.cpu().numpy()
        return e.compiled.score_matrix_oracle(X)

    def gather(self, scores: np.ndarray, valid: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """All-gather variable-length scored shards in rank order (F5)."""
        import torch

        dev = self.ctx.device if self.ctx.backend == "nccl" else torch.device("cpu")
        s = guarded_collective(all_gather_varlen, torch.as_tensor(np.asarray(scores, np.float32), device=dev),
                               self.ctx, what="score all-gather")
        v = guarded_collective(all_gather_varlen, torch.as_tensor(np.asarray(valid, np.uint8), device=dev),
                               self.ctx, what="valid all-gather")
        return s.cpu().numpy(), v.cpu().numpy().astype(bool)
