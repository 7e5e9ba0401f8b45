"""The two scoring operators of the reference, re-built around micro-batched GPU scoring.

* :class:`EvaluationFunction` — static single model (`S/api/functions/EvaluationFunction.scala:39-48`):
  the model is loaded once per subtask in ``open()``; a load failure raises
  :class:`ModelLoadingException` and fails the job.
* :class:`EvaluationCoFunction` — dynamic multi-model serving
  (`S/api/functions/EvaluationCoFunction.scala:55-133`): a control stream of Add/Del messages
  maintains the checkpointed metadata table ``ModelId → ModelInfo``; models are loaded lazily on
  the first event that needs them and cached (exact-key LRU instead of the reference's
  ``WeakHashMap[Int, _]`` keyed by hash); events for unknown models get the empty model
  (→ ``EmptyScore``); a malformed model id fails the job.

Both support two execution modes:

* ``batch_size=None`` — per-record, exactly the reference's call pattern: ``f(event, model)``
  with ``model.predict(vec)`` evaluated on the host (float64 oracle);
* ``batch_size=N`` — **micro-batching**: events are buffered; at flush time ``f`` runs once
  against a *recording* model that captures every ``predict`` input, the captured vectors are
  scored in one batch on the device (HIP kernels), and ``f`` runs again against a *replay* model
  returning those predictions. ``f`` must therefore be deterministic (no side effects besides its
  return value). Control messages, checkpoint barriers and end of input flush the buffer first,
  so the reference's ordering semantics ("event before Add → EmptyScore") hold exactly.
"""

from __future__ import annotations

import logging
from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np

from ..api.exceptions import ModelLoadingException
from ..api.managers import metadata_manager, models_manager
from ..api.pmml_model import PmmlModel
from ..api.reader import ModelReader
from ..api.vectors import as_vector
from ..domain.control import AddMessage, DelMessage, ServingMessage
from ..domain.events import event_model_id
from ..domain.model_id import ModelId, ModelInfo
from ..domain.prediction import EMPTY_PREDICTION, Prediction
from ..domain.checkpoint import STATE_NAME
from .functions import CheckpointedFunction, CoProcessFunction, Collector, FlatMapFunction

logger = logging.getLogger(__name__)


# --------------------------------------------------------------------------- record / replay models


class _RecordingModel:
    """Stands in for :class:`PmmlModel` during the capture pass: records predict() inputs."""

    def __init__(self, real: PmmlModel):
        self._real = real
        self.calls: List[Tuple[Any, Optional[float]]] = []

    def predict(self, input_vector: Any, replace_nan: Optional[float] = None) -> Prediction:
        self.calls.append((input_vector, replace_nan))
        return EMPTY_PREDICTION

    def __getattr__(self, item: str) -> Any:
        return getattr(self._real, item)


class _ReplayModel:
    def __init__(self, real: PmmlModel, preds: List[Prediction]):
        self._real = real
        self._preds = preds
        self._i = 0

    def predict(self, input_vector: Any, replace_nan: Optional[float] = None) -> Prediction:
        if self._i >= len(self._preds):
            raise RuntimeError("UDF called predict() more often in replay than in capture: UDF is not deterministic")
        p = self._preds[self._i]
        self._i += 1
        return p

    def __getattr__(self, item: str) -> Any:
        return getattr(self._real, item)


def _score_calls(model: PmmlModel, calls: List[Tuple[Any, Optional[float]]], device: Any,
                 plan_opts: dict) -> List[Prediction]:
    """Batch-score captured predict() calls (grouped by replace_nan) on ``device``."""
    if model.is_empty:
        return [EMPTY_PREDICTION] * len(calls)
    out: List[Optional[Prediction]] = [None] * len(calls)
    groups: Dict[Optional[float], List[int]] = {}
    for i, (_, rn) in enumerate(calls):
        groups.setdefault(rn, []).append(i)
    for rn, idxs in groups.items():
        vecs = [calls[i][0] for i in idxs]
        try:
            preds = model.predict_vectors(vecs, replace_nan=rn, device=device, **plan_opts)
        except Exception as e:  # noqa: BLE001 - device not lowerable etc.: fall back per record
            if device is not None:
                logger.warning("batch scoring on %s failed (%s); scoring on the host", device, e)
            preds = [model.predict(v, rn) for v in vecs]
        for i, p in zip(idxs, preds):
            out[i] = p
    return out  # type: ignore[return-value]


class _Batcher:
    """Buffers (event, model) pairs and runs the capture → batch score → replay protocol."""

    def __init__(self, f: Callable[[Any, Any], Any], batch_size: int, device: Any, plan_opts: dict):
        self.f = f
        self.batch_size = int(batch_size)
        self.device = device
        self.plan_opts = plan_opts
        self.buf: List[Tuple[Any, PmmlModel]] = []

    def add(self, event: Any, model: PmmlModel, out: Collector) -> None:
        self.buf.append((event, model))
        if len(self.buf) >= self.batch_size:
            self.flush(out)

    def flush(self, out: Collector) -> None:
        if not self.buf:
            return
        buf, self.buf = self.buf, []
        # capture pass
        recs: List[_RecordingModel] = []
        per_model: "OrderedDict[int, Tuple[PmmlModel, List[Tuple[int, int]]]]" = OrderedDict()
        all_calls: Dict[int, List[Tuple[Any, Optional[float]]]] = {}
        for ei, (ev, model) in enumerate(buf):
            rec = _RecordingModel(model)
            self.f(ev, rec)
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
            preds = _score_calls(model, all_calls[key], self.device, self.plan_opts)
            for slot, p in zip(slots, preds):
                preds_of[slot] = p
        # replay pass, in arrival order
        for ei, (ev, model) in enumerate(buf):
            preds = [preds_of[(ei, ci)] for ci in range(len(recs[ei].calls))]
            out.collect(self.f(ev, _ReplayModel(model, preds)))


# --------------------------------------------------------------------------- static operator


class EvaluationFunction(FlatMapFunction):
    """``RichFlatMapFunction[IN, OUT]`` holding one model per subtask."""

    def __init__(self, reader: ModelReader, f: Optional[Callable[[Any, PmmlModel], Any]] = None,
                 batch_size: Optional[int] = None, device: Any = None, plan_opts: Optional[dict] = None):
        self.reader = reader
        self.f = f
        self.batch_size = batch_size
        self.device = device
        self.plan_opts = plan_opts or {}
        self._evaluator: Optional[PmmlModel] = None
        self._batcher: Optional[_Batcher] = None

    @property
    def evaluator(self) -> PmmlModel:
        """Lazily loaded model (`S/api/functions/EvaluationFunction.scala:43`)."""
        if self._evaluator is None:
            self._evaluator = PmmlModel.from_reader(self.reader)
        return self._evaluator

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        try:
            model = self.evaluator
        except Exception as e:  # noqa: BLE001
            raise ModelLoadingException(str(e), e) from e
        logger.info("Model has been successfully loaded, model name: %s", model.model_name)
        if self.device is not None:
            try:
                model.compiled.plan(self.device, **self.plan_opts)  # compile once, before traffic
            except Exception as e:  # noqa: BLE001
                logger.warning("model %s is not lowerable to %s (%s); host scoring", model.model_name, self.device, e)
        if self.batch_size:
            self._batcher = _Batcher(self.f, self.batch_size, self.device, self.plan_opts)

    def flat_map(self, value: Any, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.add(value, self.evaluator, out)
        else:
            out.collect(self.f(value, self.evaluator))

    def end_of_input(self, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)

    def on_barrier(self, out: Collector) -> None:
        self.end_of_input(out)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_evaluator"] = None  # models are reloaded per subtask, never shipped
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
        else:
            self.misses += 1
        return m

    def put(self, key: ModelId, model: PmmlModel) -> None:
        self._d[key] = model
        self._d.move_to_end(key)
        while len(self._d) > self.capacity:
            self._d.popitem(last=False)

    def evict(self, keys) -> None:
        for k in keys:
            self._d.pop(k, None)

    def keys(self):
        return list(self._d.keys())

    def __contains__(self, key: ModelId) -> bool:
        return key in self._d

    def __len__(self) -> int:
        return len(self._d)


class EvaluationCoFunction(CoProcessFunction, CheckpointedFunction):
    def __init__(self, f: Optional[Callable[[Any, PmmlModel], Any]] = None, batch_size: Optional[int] = None,
                 device: Any = None, cache_capacity: int = 64, plan_opts: Optional[dict] = None):
        self.f = f
        self.batch_size = batch_size
        self.device = device
        self.cache_capacity = cache_capacity
        self.plan_opts = plan_opts or {}
        self.serving_metadata: Dict[ModelId, ModelInfo] = {}
        self.serving_models = ModelCache(cache_capacity)
        self._snapshot_metadata = None
        self._batcher: Optional[_Batcher] = None

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        if self.batch_size:
            self._batcher = _Batcher(self.f, self.batch_size, self.device, self.plan_opts)

    # -- event path (reference: `S/package.scala:111-114`)
    def model_for(self, model_id: str) -> PmmlModel:
        mid = ModelId.from_identifier(model_id)  # WrongModelIdFormat -> job failure (parity)
        m = self.serving_models.get(mid)
        if m is not None:
            return m
        return self.from_metadata(model_id)

    def process_element1(self, event: Any, ctx, out: Collector) -> None:
        model = self.model_for(event_model_id(event))
        if self._batcher is not None:
            self._batcher.add(event, model, out)
        else:
            out.collect(self.f(event, model))

    # -- control path (`S/api/functions/EvaluationCoFunction.scala:69-74`)
    def process_element2(self, control: ServingMessage, ctx, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)  # control messages are batch barriers
        self.manage_models(control)
        self.manage_metadata(control)

    def manage_models(self, control: ServingMessage) -> None:
        if isinstance(control, DelMessage):
            self.serving_models.evict(models_manager(control, self.serving_models.keys()))

    def manage_metadata(self, control: ServingMessage) -> None:
        self.serving_metadata = metadata_manager(control, self.serving_metadata)

    # -- model loading (`:98-117`)
    def load_model(self, path: str) -> PmmlModel:
        try:
            model = PmmlModel.from_reader(ModelReader(path))
        except Exception as e:  # noqa: BLE001
            raise ModelLoadingException(str(e), e) from e
        logger.info("Model has been successfully loaded, model name: %s", model.model_name)
        if self.device is not None:
            try:
                model.compiled.plan(self.device, **self.plan_opts)
            except Exception as e:  # noqa: BLE001
                logger.warning("model at %s is not lowerable to %s (%s); host scoring", path, self.device, e)
        return model

    def from_metadata(self, model_id: str) -> PmmlModel:
        mid = ModelId.from_identifier(model_id)
        info = self.serving_metadata.get(mid)
        if info is None:
            return PmmlModel.empty()
        model = self.load_model(info.path)
        self.serving_models.put(mid, model)
        return model

    loadModel = load_model  # noqa: N815
    fromMetadata = from_metadata  # noqa: N815

    # -- checkpointing (`:76-96`)
    def snapshot_state(self, context) -> None:
        self._snapshot_metadata.clear()
        self._snapshot_metadata.add(dict(self.serving_metadata))

    def initialize_state(self, context) -> None:
        self.serving_metadata = {}
        self._snapshot_metadata = context.get_operator_state_store().get_union_list_state(STATE_NAME)
        if context.is_restored():
            try:
                for snap in self._snapshot_metadata.get():
                    self.serving_metadata.update(snap)
            except Exception:  # noqa: BLE001
                logger.info("Not available state in ListState!")

    # -- flush hooks
    def end_of_input(self, out: Collector) -> None:
        if self._batcher is not None:
            self._batcher.flush(out)

    def on_barrier(self, out: Collector) -> None:
        self.end_of_input(out)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["serving_models"] = ModelCache(self.cache_capacity)
        d["_batcher"] = None
        d["_snapshot_metadata"] = None
        return d


# --------------------------------------------------------------------------- quick evaluate


def quick_udf(vec: Any, model: PmmlModel) -> Tuple[Prediction, Any]:
    """``quickEvaluate``'s UDF (`S/package.scala:138-142`)."""
    return model.predict(vec, None), vec


class QuickEvaluationFunction(FlatMapFunction):
    """Vector stream → ``(Prediction, vector)`` with native micro-batching (no capture/replay
    needed: the input *is* the vector)."""

    def __init__(self, reader: ModelReader, batch_size: Optional[int] = None, device: Any = None,
                 plan_opts: Optional[dict] = None):
        self.inner = EvaluationFunction(reader, quick_udf, None, device, plan_opts)
        self.batch_size = batch_size
        self.device = device
        self.plan_opts = plan_opts or {}
        self._buf: List[Any] = []

    def open(self, configuration: Optional[dict] = None) -> None:  # noqa: A003
        self.inner.open(configuration)

    def flat_map(self, value: Any, out: Collector) -> None:
        if not self.batch_size:
            out.collect(quick_udf(value, self.inner.evaluator))
            return
        self._buf.append(value)
        if len(self._buf) >= self.batch_size:
            self._flush(out)

    def _flush(self, out: Collector) -> None:
        if not self._buf:
            return
        buf, self._buf = self._buf, []
        preds = _score_calls(self.inner.evaluator, [(as_vector(v), None) for v in buf], self.device, self.plan_opts)
        for v, p in zip(buf, preds):
            out.collect((p, v))

    def end_of_input(self, out: Collector) -> None:
        self._flush(out)

    def on_barrier(self, out: Collector) -> None:
        self._flush(out)
