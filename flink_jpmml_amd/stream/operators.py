"""The two scoring operators of the reference, re-built around asynchronous GPU scoring.

* :class:`EvaluationFunction` — static single model (`S/api/functions/EvaluationFunction.scala:39-48`):
  the model is loaded once per subtask in ``open()`` (under ``torchrun``: parsed once on rank 0 and
  replicated to every rank); a load failure raises :class:`ModelLoadingException` and fails the job.
* :class:`EvaluationCoFunction` — dynamic multi-model serving
  (`S/api/functions/EvaluationCoFunction.scala:55-133`): a control stream of Add/Del messages
  maintains the checkpointed metadata table ``ModelId → ModelInfo``; an added model is loaded on a
  background loader thread (parse + lower never stall the event path; under ``torchrun`` the load is
  one collective: parse on rank 0, RCCL-broadcast of the compiled tensors); models are cached
  (exact-key LRU instead of the reference's ``WeakHashMap[Int, _]`` keyed by hash); events for
  unknown models get the empty model (→ ``EmptyScore``); a malformed model id fails the job; a model
  that failed to load fails the job when an event needs it (the reference's lazy-load semantics).

Element kinds, both accepted by every operator:

* **RecordBatch** (columnar fast path): ``f(batch, model)`` runs once per batch and
  ``model.predict(batch)`` returns a :class:`PredictionBatch` future — the kernel epilogue writes
  scores into pinned host memory while the operator already accepts the next batch. Results are
  emitted in order, as soon as they are ready, at most ``max_inflight`` batches behind;
* **single records** (the reference's call pattern): ``batch_size=None`` scores each record on the
  host float64 oracle exactly like the reference. ``batch_size=N`` micro-batches them:
  ``f`` runs against a *recording* model capturing every ``predict`` input, the captured vectors are
  scored as one RecordBatch on the device, and ``f`` runs again against a *replay* model. The replay
  verifies every call against the capture; an event whose UDF branched differently, or whose
  capture pass raised (e.g. ``.value.get()`` on the placeholder), is re-run per record — batching
  never changes a result. Control messages, checkpoint barriers, end of input and the
  ``max_batch_latency_ms`` timer flush the buffer, so "event before Add → EmptyScore" holds exactly.
"""

from __future__ import annotations

import collections
import logging
from collections import OrderedDict
from concurrent.futures import Future
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

import numpy as np

from ..api.batch import PredictionBatch, RecordBatch
from ..api.exceptions import ModelLoadingException
from ..api.managers import metadata_manager, models_manager
from ..api.pmml_model import PmmlModel
from ..api.reader import ModelReader
from ..api.vectors import DenseVector, SparseVector, as_vector
from ..config import ScoringConfig, merge_config
from ..domain.checkpoint import STATE_NAME
from ..domain.control import AddMessage, DelMessage, ServingMessage
from ..domain.events import event_model_id
from ..domain.model_id import ModelId, ModelInfo
from ..domain.prediction import EMPTY_PREDICTION, Prediction, Target
from ..utils.metrics import METRICS
from ..utils.profiling import prange
from .functions import CheckpointedFunction, CoProcessFunction, Collector, FlatMapFunction

logger = logging.getLogger(__name__)

DIGEST_STATE = "model-digests"


# --------------------------------------------------------------------------- shared plumbing


class _ScoringMixin:
    """Config + device + shared DevicePipeline + ordered in-flight emission of columnar results."""

    config: ScoringConfig

    def _setup(self) -> None:
        rctx = getattr(self, "runtime_context", None)
        job_cfg = getattr(rctx, "config", None)
        if self._cfg_explicit is None and job_cfg is not None:
            self.config = merge_config(job_cfg, **self._legacy)
        self.dist = getattr(rctx, "dist", None)
        local = self.dist.local_rank if self.dist is not None else 0
        self.device = self.config.resolve_device(local)
        self._pipeline = None
        self._pending: Deque[Tuple[Any, List[PredictionBatch], float]] = collections.deque()
        self._pending_timer = False

    def _pipe(self):
        if self.device is None:
            return None
        if self._pipeline is None:
            from ..runtime.engine import DevicePipeline

            self._pipeline = DevicePipeline(self.device, self.config.micro_batch, self.config.pipeline_depth,
                                            self.config.h2d_streams)
        return self._pipeline

    def _now(self) -> float:
        rctx = getattr(self, "runtime_context", None)
        return rctx.now() if rctx is not None else __import__("time").monotonic()

    # -- ordered, non-blocking emission of columnar results
    def _push(self, result: Any, out: Collector, t0: Optional[float] = None) -> None:
        """Queue a submitted result; it goes out once scored, or at ``t0`` (default: now) plus
        the latency bound, in submission order."""
        self._pending.append((result, _futures_of(result), self._now() if t0 is None else t0))
        self._emit_ready(out)
        while len(self._pending) > self.config.max_inflight:
            self._emit_one(out)
        self._arm_pending_timer(out)

    def _emit_one(self, out: Collector) -> None:
        res, _, _ = self._pending.popleft()
        if type(res) is _RecordRows:  # a per-record micro-batch: its (Prediction, vector) pairs, in order
            out.collect_many(list(zip(res.pb.predictions(), res.rows)))
        else:
            out.collect(res)

    def _emit_ready(self, out: Collector) -> None:
        while self._pending and all(f.ready for f in self._pending[0][1]):
            self._emit_one(out)

    def _drain_pending(self, out: Collector) -> None:
        while self._pending:
            self._emit_one(out)

    def _arm_pending_timer(self, out: Collector) -> None:
        lat = self.config.max_batch_latency_ms
        rctx = getattr(self, "runtime_context", None)
        if lat is None or not self._pending or self._pending_timer or rctx is None:
            return
        self._pending_timer = True
        t_first = self._pending[0][2]

        def fire(now: float) -> None:
            self._pending_timer = False
            # everything older than the bound goes out, waiting for its kernel if needed
            while self._pending and now >= self._pending[0][2] + lat / 1e3:
                self._emit_one(out)
            self._emit_ready(out)
            self._arm_pending_timer(out)

        rctx.register_timer(max(t_first + lat / 1e3, self._now()), fire)


class _RecordRows:
    """A submitted per-record micro-batch awaiting emission (QuickEvaluationFunction): the scoring
    runs while the next batch is packed; the pairs go out in arrival order once it is ready."""

    __slots__ = ("pb", "rows")

    def __init__(self, pb: PredictionBatch, rows: List[Any]):
        self.pb, self.rows = pb, rows


def _futures_of(res: Any) -> List[PredictionBatch]:
    if type(res) is _RecordRows:
        return [res.pb]
    if isinstance(res, PredictionBatch):
        return [res]
    if isinstance(res, (tuple, list)) and len(res) <= 8:
        return [x for x in res if isinstance(x, PredictionBatch)]
    return []


# --------------------------------------------------------------------------- record / replay models


class _CaptureError(Exception):
    pass


class _RecordingModel:
    """Stands in for :class:`PmmlModel` during the capture pass: records predict() inputs."""

    def __init__(self, real: PmmlModel):
        self._real = real
        self.calls: List[Tuple[Any, Optional[float]]] = []

    def predict(self, input_vector: Any, replace_nan: Optional[float] = None) -> Prediction:
        if isinstance(input_vector, RecordBatch):
            raise _CaptureError("columnar predict inside a per-record UDF")
        self.calls.append((input_vector, replace_nan))
        return EMPTY_PREDICTION

    def __getattr__(self, item: str) -> Any:
        return getattr(self._real, item)


class _ReplayMismatch(Exception):
    pass


def _same_input(a: Any, b: Any) -> bool:
    if a is b:
        return True
    try:
        return as_vector(a) == as_vector(b)
    except Exception:  # noqa: BLE001
        return False


class _ReplayModel:
    """Returns the batch-scored predictions in capture order, verifying each call's input."""

    def __init__(self, real: PmmlModel, calls: List[Tuple[Any, Optional[float]]], preds: List[Prediction]):
        self._real = real
        self._calls = calls
        self._preds = preds
        self._i = 0

    def predict(self, input_vector: Any, replace_nan: Optional[float] = None) -> Prediction:
        i = self._i
        if i >= len(self._preds):
            raise _ReplayMismatch("more predict() calls in replay than in capture")
        v0, rn0 = self._calls[i]
        if rn0 != replace_nan or not _same_input(input_vector, v0):
            raise _ReplayMismatch(f"predict() call {i} differs between capture and replay")
        self._i += 1
        return self._preds[i]

    def __getattr__(self, item: str) -> Any:
        return getattr(self._real, item)


def _score_calls(model: PmmlModel, calls: List[Tuple[Any, Optional[float]]]) -> List[Prediction]:
    """Score captured predict() calls (grouped by replace_nan) as RecordBatches on the model's
    bound scorer (device or host oracle). Device errors propagate: no silent fallback."""
    if model.is_empty:
        return [EMPTY_PREDICTION] * len(calls)
    width = len(model.active_fields)
    out: List[Optional[Prediction]] = [None] * len(calls)
    groups: Dict[Optional[float], List[int]] = {}
    for i, (_, rn) in enumerate(calls):
        groups.setdefault(rn, []).append(i)
    for rn, idxs in groups.items():
        batch = RecordBatch.from_vectors([calls[i][0] for i in idxs], width)
        preds = model.predict_records(batch, replace_nan=rn)
        for i, p in zip(idxs, preds):
            out[i] = p
    return out  # type: ignore[return-value]


class DeferredPrediction(Prediction):
    """The :class:`Prediction` a per-record UDF gets from ``model.predict`` inside a micro-batch.

    The UDF runs **exactly once per event**, when the event arrives; its ``predict`` calls are
    collected and scored together (one RecordBatch per model) when the micro-batch flushes — on
    size, latency timer, control message, barrier or end of input. A UDF that reads the score
    inside ``f`` — any access to ``prediction.value`` (``.value.get_or_else(..)``,
    ``isinstance(p.value, Score)``, ``p.value is EmptyScore``) — resolves the pending calls right
    there (a smaller batch, never a second call of ``f``), so it sees the real ``Score`` /
    ``EmptyScore`` object, as with the reference's ``case Score(v) / case EmptyScore``. UDFs that
    only return the prediction stay fully batched. The one check that cannot hold is object
    identity of the prediction itself (``p is EMPTY_PREDICTION``): compare ``p.value`` instead."""

    __slots__ = ("_batcher", "_resolved")

    def __init__(self, batcher: "_Batcher"):  # noqa: super().__init__ is not called: value is lazy
        self._batcher = batcher
        self._resolved: Optional[Prediction] = None

    def _get(self) -> Prediction:
        r = self._resolved
        if r is None:
            self._batcher.resolve()
            r = self._resolved
        return r

    @property
    def value(self) -> Target:  # type: ignore[override]
        return self._get().value

    @property
    def outputs(self):  # type: ignore[override]
        return self._get().outputs

    @property
    def resolved(self) -> bool:
        return self._resolved is not None

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, Prediction):
            return NotImplemented
        o = other._get() if isinstance(other, DeferredPrediction) else other
        return self._get() == o

    def __hash__(self) -> int:
        return hash(self._get())

    def __repr__(self) -> str:
        return repr(self._get())

    def __reduce__(self):
        return self._get().__reduce__()


class _DeferredModel:
    """Stands in for :class:`PmmlModel` inside a micro-batched UDF: ``predict`` on a vector
    registers the call and returns a :class:`DeferredPrediction`."""

    __slots__ = ("_real", "_batcher")

    def __init__(self, real: PmmlModel, batcher: "_Batcher"):
        self._real = real
        self._batcher = batcher

    def predict(self, input_vector: Any, replace_nan: Optional[float] = None):
        if isinstance(input_vector, RecordBatch) or getattr(input_vector, "ndim", 1) == 2:
            return self._real.predict(input_vector, replace_nan)
        return self._batcher.defer(self._real, input_vector, replace_nan)

    def __getattr__(self, item: str) -> Any:
        return getattr(self._real, item)


class _Batcher:
    """Micro-batches a per-record UDF (``batch_size`` set). Two modes (``ScoringConfig.udf_mode``):

    * ``deferred`` (default) — ``f(event, model)`` runs **exactly once**, as the event arrives;
      ``model.predict`` returns a :class:`DeferredPrediction`; results are emitted in arrival order
      when the batch flushes (size / latency timer / control / barrier / end), after one batched
      scoring pass per model. The reference calls ``f`` once per record
      (`S/package.scala:77-79,111-114`) — so does this mode, side effects included.
    * ``replay`` — for pure UDFs that read the score inside ``f``: ``f`` runs against a recording
      model, the captured calls are scored as one batch, and ``f`` runs again against a replay
      model that verifies every call (divergent events are re-run per record). ``f`` runs twice.
    """

    def __init__(self, owner: "_ScoringMixin", f: Callable[[Any, Any], Any], batch_size: int, mode: str = "deferred"):
        self.owner = owner
        self.f = f
        self.batch_size = int(batch_size)
        self.mode = mode
        self.buf: List[Tuple[Any, PmmlModel]] = []  # replay mode: (event, model)
        self.results: List[Any] = []  # deferred mode: UDF results, arrival order
        self.calls: List[Tuple[PmmlModel, Any, Optional[float], DeferredPrediction]] = []  # unscored
        self.first_ts: Optional[float] = None
        self._timer_armed = False

    def __len__(self) -> int:
        return len(self.results) if self.mode == "deferred" else len(self.buf)

    # -- deferred mode
    def defer(self, model: PmmlModel, vec: Any, replace_nan: Optional[float]) -> DeferredPrediction:
        dp = DeferredPrediction(self)
        self.calls.append((model, vec, replace_nan, dp))
        return dp

    def resolve(self) -> None:
        """Score every pending predict() call: one RecordBatch per (model, replace_nan)."""
        calls, self.calls = self.calls, []
        if not calls:
            return
        groups: "OrderedDict[Tuple[int, Optional[float]], list]" = OrderedDict()
        for c in calls:
            groups.setdefault((id(c[0]), c[2]), []).append(c)
        with prange("batcher.resolve"):
            for (_, rn), cs in groups.items():
                preds = _score_calls(cs[0][0], [(c[1], rn) for c in cs])
                for c, p in zip(cs, preds):
                    c[3]._resolved = p
        METRICS.inc("batcher.resolves")

    def add(self, event: Any, model: PmmlModel, out: Collector) -> None:
        if not len(self):
            self.first_ts = self.owner._now()
        if self.mode == "deferred":
            self.results.append(self.f(event, _DeferredModel(model, self)))
        else:
            self.buf.append((event, model))
        if len(self) >= self.batch_size:
            self.flush(out)
        else:
            self._arm(out)

    def add_many(self, events: List[Any], model_of: Callable[[Any], PmmlModel], out: Collector) -> None:
        """A chunk of events (deferred mode): one UDF call each, flushes at every full batch."""
        for ev in events:
            if not self.results:
                self.first_ts = self.owner._now()
            self.results.append(self.f(ev, _DeferredModel(model_of(ev), self)))
            if len(self.results) >= self.batch_size:
                self.flush(out)
        self._arm(out)

    def _arm(self, out: Collector) -> None:
        lat = self.owner.config.max_batch_latency_ms
        rctx = getattr(self.owner, "runtime_context", None)
        if lat is None or rctx is None or self._timer_armed or not len(self):
            return
        self._timer_armed = True

        def fire(now: float) -> None:
            self._timer_armed = False
            if len(self) and now >= self.first_ts + lat / 1e3:
                METRICS.inc("batcher.latency_flushes")
                self.flush(out)
            self._arm(out)

        rctx.register_timer(self.first_ts + lat / 1e3, fire)

    def flush(self, out: Collector) -> None:
        if self.mode == "deferred":
            if not self.results:
                return
            results, self.results = self.results, []
            with prange("batcher.flush"):
                self.resolve()
            out.collect_many(results)
            return
        self._flush_replay(out)

    # -- replay mode
    def _flush_replay(self, out: Collector) -> None:
        if not self.buf:
            return
        buf, self.buf = self.buf, []
        with prange("batcher.flush"):
            # capture pass
            recs: List[Optional[_RecordingModel]] = []
            per_model: "OrderedDict[int, Tuple[PmmlModel, List[Tuple[int, int]]]]" = OrderedDict()
            all_calls: Dict[int, List[Tuple[Any, Optional[float]]]] = {}
            for ei, (ev, model) in enumerate(buf):
                rec = _RecordingModel(model)
                try:
                    self.f(ev, rec)
                except Exception:  # noqa: BLE001 - e.g. .get() on the placeholder: per-record rerun
                    recs.append(None)
                    continue
                recs.append(rec)
                key = id(model)
                if key not in per_model:
                    per_model[key] = (model, [])
                    all_calls[key] = []
                for ci, call in enumerate(rec.calls):
                    per_model[key][1].append((ei, ci))
                    all_calls[key].append(call)
            # batch scoring, one batch per model
            preds_of: Dict[Tuple[int, int], Prediction] = {}
            for key, (model, slots) in per_model.items():
                preds = _score_calls(model, all_calls[key])
                for slot, p in zip(slots, preds):
                    preds_of[slot] = p
            # replay pass, in arrival order; any divergence re-runs that event per record
            for ei, (ev, model) in enumerate(buf):
                rec = recs[ei]
                res = None
                ok = False
                if rec is not None:
                    preds = [preds_of[(ei, ci)] for ci in range(len(rec.calls))]
                    try:
                        res = self.f(ev, _ReplayModel(model, rec.calls, preds))
                        ok = True
                    except _ReplayMismatch:
                        METRICS.inc("batcher.replay_mismatch")
                if not ok:
                    METRICS.inc("batcher.per_record_reruns")
                    res = self.f(ev, model)
                out.collect(res)


# --------------------------------------------------------------------------- static operator


class EvaluationFunction(FlatMapFunction, _ScoringMixin):
    """``RichFlatMapFunction[IN, OUT]`` holding one model per subtask."""

    def __init__(self, reader: ModelReader, f: Optional[Callable[[Any, PmmlModel], Any]] = None,
                 batch_size: Optional[int] = None, device: Any = None, plan_opts: Optional[dict] = None,
                 config: Optional[ScoringConfig] = None):
        self.reader = reader
        self.f = f
        self._legacy = dict(batch_size=batch_size, device=device, plan_opts=plan_opts)
        self._cfg_explicit = config
        self.config = merge_config(config, **self._legacy)
        self._evaluator: Optional[PmmlModel] = None
        self._batcher: Optional[_Batcher] = None
        self.digest: Optional[str] = None

    @property
    def batch_size(self) -> Optional[int]:
        return self.config.batch_size

    @property
    def evaluator(self) -> PmmlModel:
        """Lazily loaded model (`S/api/functions/EvaluationFunction.scala:43`)."""
        if self._evaluator is None:
            from ..runtime.loading import load_local

            lm = load_local(self.reader.source_path, getattr(self, "device", None), self.config, None)
            self._evaluator, self.digest = lm.model, lm.sha256
        return self._evaluator

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        from ..runtime.loading import load_replicated

        self._setup()
        try:
            lm = load_replicated(self.reader.source_path, self.dist, self.device, self.config, self._pipe())
        except ModelLoadingException:
            raise
        except Exception as e:  # noqa: BLE001
            raise ModelLoadingException(str(e), e) from e
        self._evaluator, self.digest = lm.model, lm.sha256
        logger.info("Model has been successfully loaded, model name: %s", lm.model.model_name)
        if self.config.batch_size:
            self._batcher = _Batcher(self, self.f, self.config.batch_size, self.config.udf_mode)

    def flat_map(self, value: Any, out: Collector) -> None:
        if isinstance(value, RecordBatch):
            with prange("evaluate.batch"):
                self._push(self.f(value, self.evaluator), out)
        elif self._batcher is not None:
            self._batcher.add(value, self.evaluator, out)
        else:
            out.collect(self.f(value, self.evaluator))

    def flat_map_many(self, values: List[Any], out: Collector) -> None:
        """Chunked delivery of per-record events (same results as element-wise)."""
        if any(type(v) is RecordBatch for v in values):
            for v in values:
                self.flat_map(v, out)
            return
        model = self.evaluator
        b = self._batcher
        if b is None:
            f = self.f
            out.collect_many([f(v, model) for v in values])
        elif b.mode == "deferred":
            b.add_many(values, lambda ev: model, out)
        else:
            for v in values:
                b.add(v, model, out)

    def end_of_input(self, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)
        self._drain_pending(out)

    def on_barrier(self, out: Collector) -> None:
        self.end_of_input(out)

    def checkpoint_models(self) -> Dict[str, dict]:
        return {f"static:{self.reader.source_path}": {"path": self.reader.source_path, "sha256": self.digest}} \
            if self.digest else {}

    def __getstate__(self):
        d = dict(self.__dict__)
        for k in ("_evaluator", "_batcher", "_pipeline", "_pending", "dist", "runtime_context"):
            d.pop(k, None)  # models are reloaded per subtask, never shipped
        d["_evaluator"] = None
        d["_batcher"] = None
        return d


# --------------------------------------------------------------------------- dynamic operator


class ModelCache:
    """Exact-key LRU cache ``ModelId → PmmlModel`` (replaces the reference's GC-evictable
    ``WeakHashMap[Int, PmmlModel]`` keyed by a 32-bit hash)."""

    def __init__(self, capacity: int = 64):
        self.capacity = capacity
        self._d: "OrderedDict[ModelId, PmmlModel]" = OrderedDict()
        self.hits = 0
        self.misses = 0

    def get(self, key: ModelId) -> Optional[PmmlModel]:
        m = self._d.get(key)
        if m is not None:
            self._d.move_to_end(key)
            self.hits += 1
            METRICS.inc("model_cache.hits")
        else:
            self.misses += 1
            METRICS.inc("model_cache.misses")
        return m

    def put(self, key: ModelId, model: PmmlModel) -> None:
        self._d[key] = model
        self._d.move_to_end(key)
        while len(self._d) > self.capacity:
            self._d.popitem(last=False)
            METRICS.inc("model_cache.evictions")

    def evict(self, keys) -> None:
        for k in keys:
            self._d.pop(k, None)

    def keys(self):
        return list(self._d.keys())

    def __contains__(self, key: ModelId) -> bool:
        return key in self._d

    def __len__(self) -> int:
        return len(self._d)


class EvaluationCoFunction(CoProcessFunction, CheckpointedFunction, _ScoringMixin):
    def __init__(self, f: Optional[Callable[[Any, PmmlModel], Any]] = None, batch_size: Optional[int] = None,
                 device: Any = None, cache_capacity: Optional[int] = None, plan_opts: Optional[dict] = None,
                 config: Optional[ScoringConfig] = None):
        self.f = f
        self._legacy = dict(batch_size=batch_size, device=device, cache_capacity=cache_capacity,
                            plan_opts=plan_opts)
        self._cfg_explicit = config
        self.config = merge_config(config, **self._legacy)
        self.serving_metadata: Dict[ModelId, ModelInfo] = {}
        self.serving_models = ModelCache(self.config.cache_capacity)
        self.digests: Dict[ModelId, str] = {}
        self._snapshot_metadata = None
        self._snapshot_digests = None
        self._batcher: Optional[_Batcher] = None
        self._loading: Dict[ModelId, Future] = {}
        self._loader = None
        self.dist = None
        self.device = None
        self._pipeline = None
        self._pending = collections.deque()
        self._restored_digests: Dict[ModelId, str] = {}
        self._by_str: Dict[str, PmmlModel] = {}
        self.grouped = False  # quick mode: columnar batches -> (PredictionBatch, RecordBatch), any id mix
        self._grouped_scorer = None

    @property
    def batch_size(self) -> Optional[int]:
        return self.config.batch_size

    @property
    def cache_capacity(self) -> int:
        return self.config.cache_capacity

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        self._setup()
        self.serving_models.capacity = self.config.cache_capacity
        if self.config.batch_size:
            self._batcher = _Batcher(self, self.f, self.config.batch_size, self.config.udf_mode)
        # models of a restored checkpoint are re-loaded (and re-replicated) right away
        if self.config.async_load or self._distributed:
            for mid, info in self.serving_metadata.items():
                self._schedule_load(mid, info.path)

    @property
    def _distributed(self) -> bool:
        return self.dist is not None and self.dist.is_distributed

    # -- loading
    def _load_fn(self, path: str):
        from ..runtime.loading import load_replicated

        return load_replicated(path, self.dist, self.device, self.config, self._pipe())

    def _schedule_load(self, mid: ModelId, path: str) -> None:
        from ..runtime.loading import ModelLoader

        if self._loader is None:
            self._loader = ModelLoader(self._load_fn, name=f"model-loader-{id(self):x}")
        self._loading[mid] = self._loader.submit(path)

    def _accept_loaded(self, mid: ModelId, lm) -> PmmlModel:
        pinned = self._restored_digests.get(mid)
        if pinned is not None and pinned != lm.sha256:
            raise ModelLoadingException(f"model {mid} at {lm.path} changed since the checkpoint "
                                        f"(sha256 {lm.sha256[:12]}… != {pinned[:12]}…)")
        self.digests[mid] = lm.sha256
        self.serving_models.put(mid, lm.model)
        logger.info("Model has been successfully loaded, model name: %s", lm.model.model_name)
        return lm.model

    def load_model(self, path: str) -> PmmlModel:
        """Synchronous local load (`S/api/functions/EvaluationCoFunction.scala:98-104`)."""
        from ..runtime.loading import load_local

        try:
            lm = load_local(path, self.device, self.config, self._pipe() if self.device is not None else None)
        except ModelLoadingException:
            raise
        except Exception as e:  # noqa: BLE001
            raise ModelLoadingException(str(e), e) from e
        logger.info("Model has been successfully loaded, model name: %s", lm.model.model_name)
        self._last_digest = lm.sha256
        return lm.model

    # -- event path (reference: `S/package.scala:111-114`)
    def model_for(self, model_id: str) -> PmmlModel:
        mid = ModelId.from_identifier(model_id)  # WrongModelIdFormat -> job failure (parity)
        m = self.serving_models.get(mid)
        if m is not None:
            return m
        fut = self._loading.pop(mid, None)
        if fut is not None and mid in self.serving_metadata:
            try:
                with prange("model.wait_load"):
                    lm = fut.result()
            except ModelLoadingException:
                raise
            except Exception as e:  # noqa: BLE001
                raise ModelLoadingException(str(e), e) from e
            return self._accept_loaded(mid, lm)
        return self.from_metadata(model_id)

    def _model_of_event(self, event: Any) -> PmmlModel:
        """``model_for`` with a per-id-string memo (cleared by every control message): a stream of
        events for the same few models skips the id parse and the cache lookup."""
        key = event_model_id(event)
        m = self._by_str.get(key)
        if m is None:
            m = self.model_for(key)
            if not m.is_empty:
                self._by_str[key] = m
        return m

    def process_elements1(self, events: List[Any], ctx, out: Collector) -> None:
        """Chunked delivery of per-record events (same results as element-wise)."""
        b = self._batcher
        if any(type(e) is RecordBatch for e in events) or (b is not None and b.mode != "deferred"):
            for e in events:
                self.process_element1(e, ctx, out)
            return
        if b is None:
            f = self.f
            out.collect_many([f(e, self._model_of_event(e)) for e in events])
        else:
            b.add_many(events, self._model_of_event, out)

    def score_mixed(self, batch: RecordBatch) -> PredictionBatch:
        """One row-order :class:`PredictionBatch` for a columnar batch whose rows may name different
        models (``model_ids``): row ``i`` equals ``model_for(id_i).predict(batch.vector(i))``.
        Device models are scored in one grouped pass (one H2D, device-side grouping, a launch per
        model present: ``runtime/grouped.py``); anything else is split per model and merged."""
        keep = self.config.device_mirror
        if not batch.has_model_ids:
            return self.model_for(batch.model_id).predict_records(batch, keep_device=keep)
        codes, keys = batch.id_codes()
        models = [self.model_for(k) for k in keys]  # WrongModelIdFormat fails the job (parity)
        if len(models) == 1:
            return models[0].predict_records(batch, keep_device=keep)
        from ..runtime.engine import NullScorer
        from ..runtime.grouped import GroupedScorer, NotGroupable, groupable

        width = batch.n_features
        scorers = [NullScorer(width) if m.is_empty or len(m.active_fields) != width else m.scorer for m in models]
        pipe = self._pipe()
        if pipe is not None and groupable(scorers, width) is None and \
                all(getattr(sc, "pipe", pipe) is pipe for sc in scorers):
            if self._grouped_scorer is None:
                self._grouped_scorer = GroupedScorer(pipe, max_inflight=self.config.max_inflight)
            try:
                return self._grouped_scorer.submit(batch, codes, scorers, keep_device=keep)
            except NotGroupable:  # pragma: no cover - groupable() checked the same conditions
                pass
        # split path: per-model predict + merge. Rows of an empty model or of one whose active
        # fields differ from the batch width are EmptyScore, as on the grouped path (NullScorer).
        # The merged batch has no device mirrors: a device GatherSink takes its host path for it.
        METRICS.inc("grouped.split_batches")
        n = len(batch)
        s = np.full(n, np.nan, dtype=np.float32)
        v = np.zeros(n, dtype=bool)
        for sub in batch.split_by_model():
            m = self.model_for(sub.model_id)
            if m.is_empty or len(m.active_fields) != width:
                continue
            pb = m.predict_records(sub)
            s[sub.row_index] = pb.scores
            v[sub.row_index] = pb.valid
        return PredictionBatch.from_arrays(s, v).masked(batch.size_ok())

    def process_element1(self, event: Any, ctx, out: Collector) -> None:
        if isinstance(event, RecordBatch) and self.grouped:
            with prange("evaluate.grouped"):
                self._push((self.score_mixed(event), event), out)
            return
        if isinstance(event, RecordBatch):
            for sub in event.split_by_model():
                model = self.model_for(sub.model_id)
                with prange("evaluate.batch"):
                    self._push(self.f(sub, model), out)
            return
        model = self.model_for(event_model_id(event))
        if self._batcher is not None:
            self._batcher.add(event, model, out)
        else:
            out.collect(self.f(event, model))

    # -- control path (`S/api/functions/EvaluationCoFunction.scala:69-74`)
    def process_element2(self, control: ServingMessage, ctx, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)  # control messages are batch barriers
        self._drain_pending(out)
        self._by_str.clear()
        self.manage_models(control)
        known = control.model_id in self.serving_metadata
        self.manage_metadata(control)
        METRICS.inc(f"control.{type(control).__name__}")
        if isinstance(control, AddMessage) and not known and (self.config.async_load or self._distributed):
            self._schedule_load(control.model_id, control.path)

    def manage_models(self, control: ServingMessage) -> None:
        if isinstance(control, DelMessage):
            self.serving_models.evict(models_manager(control, self.serving_models.keys()))
            self._loading.pop(control.model_id, None)  # a running load finishes and is dropped
            self.digests.pop(control.model_id, None)

    def manage_metadata(self, control: ServingMessage) -> None:
        self.serving_metadata = metadata_manager(control, self.serving_metadata)

    def from_metadata(self, model_id: str) -> PmmlModel:
        mid = ModelId.from_identifier(model_id)
        info = self.serving_metadata.get(mid)
        if info is None:
            METRICS.inc("scoring.unknown_model_events")
            return PmmlModel.empty()
        from ..runtime.loading import load_local

        try:  # lazy (non-collective) load: evicted models, or async_load=False
            lm = load_local(info.path, self.device, self.config, self._pipe() if self.device is not None else None)
        except ModelLoadingException:
            raise
        except Exception as e:  # noqa: BLE001
            raise ModelLoadingException(str(e), e) from e
        return self._accept_loaded(mid, lm)

    loadModel = load_model  # noqa: N815
    fromMetadata = from_metadata  # noqa: N815

    # -- checkpointing (`:76-96`)
    def snapshot_state(self, context) -> None:
        self._snapshot_metadata.clear()
        self._snapshot_metadata.add(dict(self.serving_metadata))
        self._snapshot_digests.clear()
        self._snapshot_digests.add({str(k): v for k, v in self.digests.items() if k in self.serving_metadata})

    def initialize_state(self, context) -> None:
        self.serving_metadata = {}
        store = context.get_operator_state_store()
        self._snapshot_metadata = store.get_union_list_state(STATE_NAME)
        self._snapshot_digests = store.get_union_list_state(DIGEST_STATE)
        if context.is_restored():
            try:
                for snap in self._snapshot_metadata.get():
                    self.serving_metadata.update(snap)
                for snap in self._snapshot_digests.get():
                    self._restored_digests.update({ModelId.from_identifier(k): v for k, v in snap.items()})
            except Exception:  # noqa: BLE001
                logger.info("Not available state in ListState!")

    def checkpoint_models(self) -> Dict[str, dict]:
        return {str(mid): {"path": info.path, "sha256": self.digests.get(mid) or self._restored_digests.get(mid)}
                for mid, info in self.serving_metadata.items()}

    # -- flush hooks
    def end_of_input(self, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)
        self._drain_pending(out)

    def on_barrier(self, out: Collector) -> None:
        self.end_of_input(out)

    def close(self) -> None:
        if self._loader is not None:
            self._loader.close(wait=True)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["serving_models"] = ModelCache(self.config.cache_capacity)
        for k in ("_batcher", "_snapshot_metadata", "_snapshot_digests", "_loader", "_pipeline", "dist",
                  "runtime_context"):
            d[k] = None
        d["_loading"] = {}
        d["_pending"] = collections.deque()
        d["_by_str"] = {}
        return d


# --------------------------------------------------------------------------- quick evaluate


def quick_udf(vec: Any, model: PmmlModel) -> Tuple[Any, Any]:
    """``quickEvaluate``'s UDF (`S/package.scala:138-142`): ``(Prediction, vector)`` per record,
    ``(PredictionBatch, RecordBatch)`` per columnar batch."""
    return model.predict(vec, None), vec


class QuickEvaluationFunction(FlatMapFunction, _ScoringMixin):
    """Vector stream → ``(Prediction, vector)``; RecordBatch stream → ``(PredictionBatch,
    RecordBatch)``. Per-record vectors are micro-batched natively when ``batch_size`` is set (no
    capture/replay needed: the input *is* the vector)."""

    def __init__(self, reader: ModelReader, batch_size: Optional[int] = None, device: Any = None,
                 plan_opts: Optional[dict] = None, config: Optional[ScoringConfig] = None):
        self.inner = EvaluationFunction(reader, quick_udf, None, device, plan_opts, config)
        self._legacy = dict(batch_size=batch_size, device=device, plan_opts=plan_opts)
        self._cfg_explicit = config
        self.config = merge_config(config, **self._legacy)
        self._buf: List[Any] = []
        self._first_ts: Optional[float] = None
        self._timer = False

    @property
    def batch_size(self) -> Optional[int]:
        return self.config.batch_size

    def set_runtime_context(self, ctx) -> None:
        super().set_runtime_context(ctx)
        self.inner.set_runtime_context(ctx)

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        self._setup()
        self.inner._cfg_explicit = self._cfg_explicit
        self.inner._legacy = dict(self._legacy, batch_size=None)
        self.inner.open(configuration)
        self.inner.config = self.inner.config.replace(batch_size=None)

    def flat_map(self, value: Any, out: Collector) -> None:
        if isinstance(value, RecordBatch):
            with prange("quick_evaluate.batch"):
                self._push((self.inner.evaluator.predict_records(value, keep_device=self.config.device_mirror),
                            value), out)
            return
        if not self.config.batch_size:
            out.collect(quick_udf(value, self.inner.evaluator))
            return
        if not self._buf:
            self._first_ts = self._now()
        self._buf.append(value)
        if len(self._buf) >= self.config.batch_size:
            self._flush(out)
        else:
            self._arm(out)

    def flat_map_many(self, values: List[Any], out: Collector) -> None:
        """Chunked delivery: per-record vectors are appended in bulk and flushed per full batch."""
        has_rb = RecordBatch in set(map(type, values))
        if not self.config.batch_size or has_rb:
            if not self.config.batch_size and not has_rb:
                model = self.inner.evaluator
                out.collect_many([quick_udf(v, model) for v in values])
                return
            for v in values:
                self.flat_map(v, out)
            return
        bs = self.config.batch_size
        i, n = 0, len(values)
        while i < n:
            if not self._buf:
                self._first_ts = self._now()
            take = min(n - i, bs - len(self._buf))
            self._buf.extend(values[i:i + take] if (i or take < n) else values)
            i += take
            if len(self._buf) >= bs:
                self._flush(out)
        self._arm(out)

    def _arm(self, out: Collector) -> None:
        lat = self.config.max_batch_latency_ms
        rctx = getattr(self, "runtime_context", None)
        if lat is None or rctx is None or self._timer or not self._buf:
            return
        self._timer = True

        def fire(now: float) -> None:
            self._timer = False
            if self._buf and now >= self._first_ts + lat / 1e3:
                METRICS.inc("batcher.latency_flushes")
                self._flush(out)
                self._drain_pending(out)  # the latency bound is due: out now, waiting for the kernel
            self._arm(out)

        rctx.register_timer(self._first_ts + lat / 1e3, fire)

    def _flush(self, out: Collector) -> None:
        if not self._buf:
            return
        buf, self._buf = self._buf, []
        model = self.inner.evaluator
        with prange("quick_evaluate.flush"):
            batch = RecordBatch.from_vectors(buf, len(model.active_fields))
            # submitted, not awaited: the pairs go out when the kernel is done (or at the latency
            # bound / barrier / end of input), so the next batch packs while this one scores
            self._push(_RecordRows(model.predict_records(batch), buf), out, t0=self._first_ts)

    def end_of_input(self, out: Collector) -> None:
        self._flush(out)
        self._drain_pending(out)

    def on_barrier(self, out: Collector) -> None:
        self.end_of_input(out)

    def checkpoint_models(self) -> Dict[str, dict]:
        return self.inner.checkpoint_models()

    def __getstate__(self):
        d = dict(self.__dict__)
        for k in ("_pipeline", "_pending", "dist", "runtime_context"):
            d.pop(k, None)
        d["_buf"] = []
        return d


# --------------------------------------------------------------------------- event -> batch adapter


def _row_of(x: Any) -> Any:
    data = getattr(x, "data", None)
    if data is not None and not isinstance(x, SparseVector):
        return data
    if isinstance(x, SparseVector):
        return x.to_dense_array()
    return x


class ToBatchesFunction(FlatMapFunction):
    """``DataStream.to_batches``: accumulates per-record events into RecordBatches (see there)."""

    def __init__(self, extract: Optional[Callable[[Any], Any]], batch_rows: int,
                 model_id: Optional[Callable[[Any], str]], keep_events: bool, max_latency_ms: Optional[float]):
        self.extract = extract
        self.batch_rows = int(batch_rows)
        self.model_id = model_id
        self.keep_events = bool(keep_events)
        self.max_latency_ms = max_latency_ms
        self._rows: List[Any] = []
        self._events: List[Any] = []
        self._first: Optional[float] = None
        self._timer = False
        self._offset = 0

    def _now(self) -> float:
        rctx = getattr(self, "runtime_context", None)
        return rctx.now() if rctx is not None else __import__("time").monotonic()

    def flat_map(self, value: Any, out: Collector) -> None:
        self.flat_map_many([value], out)

    def flat_map_many(self, values: List[Any], out: Collector) -> None:
        ex = self.extract
        i, n = 0, len(values)
        while i < n:
            if not self._events:
                self._first = self._now()
            take = min(n - i, self.batch_rows - len(self._events))
            part = values[i:i + take] if (i or take < n) else values
            self._rows.extend(map(ex, part) if ex is not None else map(_row_of, part))
            self._events.extend(part)
            i += take
            if len(self._events) >= self.batch_rows:
                self._emit(out)
        self._arm(out)

    def _emit(self, out: Collector) -> None:
        if not self._events:
            return
        rows, events = self._rows, self._events
        self._rows, self._events = [], []
        rows = [_row_of(r) if isinstance(r, (DenseVector, SparseVector)) else r for r in rows] \
            if rows and isinstance(rows[0], (DenseVector, SparseVector)) else rows
        X = None
        if rows and type(rows[0]) is np.ndarray and rows[0].ndim == 1:
            w = rows[0].shape[0]
            if all(type(r) is np.ndarray and r.shape == (w,) for r in rows):
                X = np.concatenate(rows).astype(np.float64, copy=False).reshape(len(rows), w)
        if X is None:
            X = np.asarray(rows, dtype=np.float64)
        if X.ndim != 2:
            raise ValueError(f"to_batches: extract() must give one feature row per event, got shape {X.shape}")
        ids = [self.model_id(e) for e in events] if self.model_id is not None else None
        uniq = set(ids) if ids is not None else None
        b = RecordBatch(X, model_id=next(iter(uniq)) if uniq is not None and len(uniq) == 1 else None,
                        model_ids=ids if uniq is not None and len(uniq) > 1 else None,
                        payload=events if self.keep_events else None, offset=self._offset)
        self._offset += len(events)
        METRICS.inc("to_batches.batches")
        out.collect(b)

    def _arm(self, out: Collector) -> None:
        lat = self.max_latency_ms
        rctx = getattr(self, "runtime_context", None)
        if lat is None or rctx is None or self._timer or not self._events:
            return
        self._timer = True

        def fire(now: float) -> None:
            self._timer = False
            if self._events and now >= self._first + lat / 1e3:
                self._emit(out)
            self._arm(out)

        rctx.register_timer(self._first + lat / 1e3, fire)

    def end_of_input(self, out: Collector) -> None:
        self._emit(out)

    def on_barrier(self, out: Collector) -> None:
        self._emit(out)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_rows"], d["_events"] = [], []
        d.pop("runtime_context", None)
        return d
