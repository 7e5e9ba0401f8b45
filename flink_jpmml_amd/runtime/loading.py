"""Model loading for the streaming operators: read → parse → lower → bind, locally or
**parse-once-and-replicate** across GPU ranks, synchronously or on a background loader thread.

Reference behaviour: every Flink subtask reads and parses the PMML itself, lazily on the first
event that needs it (`S/api/functions/EvaluationFunction.scala:43`,
`S/api/functions/EvaluationCoFunction.scala:98-117`); a failure is fatal
(:class:`ModelLoadingException`). Here:

* :func:`load_local` — this process reads, parses (and lowers to its GPU);
* :func:`load_replicated` — a collective over the ``model`` process group: rank 0 reads, parses
  and lowers once; the document bytes and the compiled device tensors travel to every rank
  (RCCL broadcast over xGMI). Other ranks never parse unless a host-only path asks
  for the IR (:class:`LazyCompiled` parses on first use);
* :class:`ModelLoader` — one background thread per operator instance executing load tasks in
  submission order, so a new model's ≈seconds of parse + lowering never stall the event path
  (an event only waits when it needs that very model). Under data parallelism every rank submits
  the same Add messages in the same order, so the loader threads' collectives match.

Every load records the document's sha256 (checkpoint manifests pin it) and its duration
(``model.load_ms`` histogram).
"""

from __future__ import annotations

import hashlib
import logging
import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass
from typing import Any, Callable, Optional

from ..api.evaluator import Evaluator
from ..api.exceptions import ModelLoadingException
from ..api.pmml_model import PmmlModel
from ..api.reader import ModelReader
from ..utils.metrics import METRICS
from ..utils.profiling import prange

logger = logging.getLogger(__name__)


@dataclass
class LoadedModel:
    model: PmmlModel
    sha256: str
    path: str
    load_ms: float


class LazyCompiled:
    """Stand-in for :class:`CompiledPmml` on ranks that received a replicated model: the field
    lists come from rank 0; the document is parsed only if something needs the IR (per-record
    host predict, host fallback)."""

    def __init__(self, text: str, source: Optional[str], header: dict):
        self._text = text
        self._source = source
        self._real = None
        self._lock = threading.Lock()
        self.active_fields = list(header["active_fields"])
        self.target_fields = list(header["target_fields"])
        self.output_fields = list(header.get("output_fields", []))
        self.model_name = header.get("model_name")
        self.source = source

    @property
    def n_features(self) -> int:
        return len(self.active_fields)

    def _materialise(self):
        with self._lock:
            if self._real is None:
                from .compiled import CompiledPmml

                self._real = CompiledPmml.from_string(self._text, source=self._source)
            return self._real

    def __getattr__(self, item: str) -> Any:
        if item.startswith("__"):
            raise AttributeError(item)
        return getattr(self._materialise(), item)


def _header(compiled) -> dict:
    return {"active_fields": list(compiled.active_fields), "target_fields": list(compiled.target_fields),
            "output_fields": list(getattr(compiled, "output_fields", [])), "model_name": compiled.model_name}


def _read(path: str) -> bytes:
    """The document's bytes (UTF-8): parsed directly by the streaming scanner for large models and
    hashed as-is — no 2× decode/encode of a several-hundred-MB string."""
    return ModelReader(path).read_bytes()


def load_local(path: str, device: Any = None, config: Any = None, pipeline: Any = None) -> LoadedModel:
    """Read + parse + lower + bind in this process. Raises :class:`ModelLoadingException`."""
    from .compiled import CompiledPmml

    t0 = time.perf_counter()
    with prange("model.load"):
        try:
            text = _read(path)
            compiled = CompiledPmml.from_string(text, source=path)
        except Exception as e:  # noqa: BLE001 - any read/parse failure is a load failure
            raise ModelLoadingException(f"{type(e).__name__}: {e}", e) from e
        model = PmmlModel(Evaluator.apply(compiled)).bind(device, config, pipeline)
        _sync_device(device)
    ms = (time.perf_counter() - t0) * 1e3
    METRICS.observe("model.load_ms", ms)
    METRICS.inc("model.loads")
    return LoadedModel(model, hashlib.sha256(text).hexdigest(), path, ms)


def _sync_device(device) -> None:
    """Plans are built with copies on this thread's current stream: finish them before another
    thread's streams use the tensors."""
    if device is not None:
        import torch

        if torch.cuda.is_available():
            torch.cuda.current_stream(device).synchronize()


def load_replicated(path: str, ctx, device: Any = None, config: Any = None, pipeline: Any = None) -> LoadedModel:
    """Collective over ``ctx``'s ``model`` group (every rank calls it, in the same order): rank 0
    reads, parses and lowers; ranks receive the document and the compiled device tensors."""
    if ctx is None or not ctx.is_distributed:
        return load_local(path, device, config, pipeline)
    from ..config import ScoringConfig
    from ..parallel.dist import broadcast_object, broadcast_tensors
    from .compiled import CompiledPmml
    from .plans import DevicePlan


    cfg = config or ScoringConfig()
    g = ctx.group("model")
    # F2 ordering rule: the header / error / plan-metadata handshake runs on the
    # loader thread's own GLOO group, so ranks 1..N-1 block on the host while rank 0 reads, parses
    # and lowers (seconds for a large document) -- no device collective spins on the GPU meanwhile.
    # The RCCL payload broadcast on ``model`` is issued only after it, when every rank is ready.
    gh = ctx.groups.get("model_ctrl") or ctx.group("ctrl")
    t0 = time.perf_counter()
    compiled = plan = None
    head: dict = {}
    with prange("model.load_replicated"):
        if ctx.is_root:
            try:
                text = _read(path)
                compiled = CompiledPmml.from_string(text, source=path)
                head = {"text": text, "header": _header(compiled)}
            except Exception as e:  # noqa: BLE001 - the leader reports, every rank fails alike
                head = {"err": f"{type(e).__name__}: {e}"}
            if "err" not in head and device is not None and compiled.target_fields:
                try:
                    with prange("model.lower"):
                        plan = compiled.plan(device, **cfg.lowering_opts())
                    head["plan_meta"] = plan.export_state()[0]
                except Exception as e:  # noqa: BLE001 - reported to every rank before the broadcast
                    # (a lowering error escaping here would leave the peers blocked in the
                    # broadcast until the timeout): all ranks then fall back or fail alike
                    plan = None
                    head["lower_error"] = f"{type(e).__name__}: {e}"
        head = broadcast_object(head, ctx, group=gh)
        if "err" in head:
            raise ModelLoadingException(f"model at {path}: {head['err']}")
        meta = head.get("plan_meta")
        if meta is not None and device is not None:
            tensors = plan.export_state()[1] if ctx.is_root else None
            got = broadcast_tensors(tensors, meta["__tensors__"], ctx, group=g)
            METRICS.inc("dist.bytes_broadcast", sum(t.numel() * t.element_size() for t in got.values()))
            if not ctx.is_root:
                plan = DevicePlan.from_state(meta, got, device)
        if not ctx.is_root:
            compiled = LazyCompiled(head["text"], path, head["header"])
        model = PmmlModel(Evaluator.apply(compiled))
        from .engine import make_scorer

        model._scorer = make_scorer(compiled, device, cfg, pipeline, plan=plan,
                                    lower_error=head.get("lower_error"))
        _sync_device(device)
    ms = (time.perf_counter() - t0) * 1e3
    METRICS.observe("model.load_ms", ms)
    METRICS.inc("model.loads_replicated")
    return LoadedModel(model, hashlib.sha256(head["text"]).hexdigest(), path, ms)


class ModelLoader:
    """Single background thread running load tasks in submission order. ``submit`` returns a
    :class:`concurrent.futures.Future` of :class:`LoadedModel` (or the load exception)."""

    def __init__(self, load_fn: Callable[[str], LoadedModel], name: str = "model-loader"):
        self._fn = load_fn
        self._q: "queue.Queue" = queue.Queue()
        self._t = threading.Thread(target=self._run, name=name, daemon=True)
        self._started = False
        self._closed = False

    def submit(self, path: str) -> Future:
        if not self._started:
            self._t.start()
            self._started = True
        fut: Future = Future()
        self._q.put((path, fut))
        return fut

    def _run(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            path, fut = item
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                fut.set_result(self._fn(path))
            except BaseException as e:  # noqa: BLE001 - delivered to the waiting event
                fut.set_exception(e)

    def close(self, wait: bool = True) -> None:
        if self._started and not self._closed:
            self._closed = True
            self._q.put(None)
            if wait:
                self._t.join(timeout=600)


__all__ = ["LazyCompiled", "LoadedModel", "ModelLoader", "load_local", "load_replicated"]
