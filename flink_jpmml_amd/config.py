"""Scoring configuration: one dataclass for every knob of the streaming scorer.

The reference has no configuration object — its only parameters are API arguments
(``ModelReader(path)``, ``predict(vec, replaceNan)``) and the example jobs' ``ParameterTool`` flags
(`E/util/DynamicParams.scala:28-43`). The MI355X engine has real knobs (micro-batch size, latency
bound, device placement, leaf/weight precision, cache size, …); they live here and are accepted by
every DSL entry point (``config=``) and by the example CLIs (same flag names where they overlap).

    cfg = ScoringConfig(batch_size=65536, max_batch_latency_ms=5.0, device="cuda")
    stream.quick_evaluate(ModelReader(path), config=cfg)

``ScoringConfig.from_env()`` reads ``FJA_*`` environment variables (``FJA_BATCH_SIZE``,
``FJA_MAX_BATCH_LATENCY_MS``, ``FJA_DEVICE``, ``FJA_PRECISION``, ``FJA_FALLBACK``, …).
"""

from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Sequence

PRECISIONS = ("fp32", "bf16", "fp8")
FALLBACKS = ("host", "warn", "error")


@dataclass
class ScoringConfig:
    # -- micro-batching of per-record streams (capture/replay path)
    batch_size: Optional[int] = None
    """Flush a per-record micro-batch once it holds this many records (``None`` = score each record
    as it arrives, exactly the reference's call pattern)."""
    udf_mode: str = "deferred"
    """How a micro-batched per-record UDF is run: ``deferred`` — exactly once per event, its
    ``predict`` calls resolved when the batch is scored; ``replay`` — capture, batch score, replay
    (the UDF runs twice: pure UDFs that read the score inside ``f`` batch fully)."""
    max_batch_latency_ms: Optional[float] = None
    """Flush a non-empty micro-batch once its oldest record has waited this long (size-or-time
    trigger). ``None`` = size, control message, checkpoint barrier or end of input only."""

    # -- device placement and precision
    device: Any = "auto"
    """HIP device for model kernels (``"cuda"``, ``"cuda:3"``); ``"auto"`` (default) = the rank's
    GPU when one is visible, else the host; ``None`` / ``"cpu"`` = host float64 oracle. Under
    ``torchrun`` every rank uses its own GPU (``cuda:LOCAL_RANK``) for ``"cuda"`` / ``"auto"``."""
    device_ids: Optional[Sequence[int]] = None
    """Explicit GPU per rank (``device_ids[local_rank]``), overrides the ``LOCAL_RANK`` default."""
    precision: str = "fp32"
    """``fp32`` (exact-fp32 kernels, default), ``bf16`` (NeuralNetwork GEMMs on bf16 MFMA; other
    families stay fp32), ``fp8`` (tree leaves / calibrator in OCP e4m3; NeuralNetwork on bf16).
    Split thresholds and every decision stay fp32 always."""
    fallback: str = "warn"
    """What happens when a model cannot be lowered to the device: ``host`` — score on the host
    oracle (batched, vectorised) and count ``scoring.host_fallback``; ``warn`` — the same plus one
    WARNING per model; ``error`` — fail the model load (strict production setting)."""

    host_threads: int = 0
    """Worker threads of the native host tree walk (``fallback="host"`` models, CPU-only ranks,
    direct CPU ``predict_batch``); 0 = ``FJA_HOST_THREADS`` or 1. Results do not depend on it."""

    # -- columnar (RecordBatch) pipeline
    micro_batch: int = 1 << 19
    """Rows per device kernel launch when a RecordBatch is split (H2D / kernel overlap)."""
    pipeline_depth: int = 3
    """Device input slots of the H2D → kernel ring (copy of batch i+1 overlaps kernel i)."""
    h2d_streams: int = 0
    """Copy streams each micro-batch's host→device transfer is split over (concurrent copy
    engines); 0 = calibrate 1 vs 2 on the first copy and keep the faster (boxes differ)."""
    max_inflight: int = 4
    """Scored batches an operator keeps in flight before it waits for the oldest (backpressure)."""
    metrics_port: int = 0
    """> 0: every rank serves its metrics in the Prometheus text format on ``GET /metrics`` at
    ``metrics_port + rank`` (127.0.0.1) while a job runs (``utils/metrics.py``)."""
    graph_max_rows: int = 16384
    """Micro-batches of at most this many rows run multi-kernel plans (wide NeuralNetworks,
    segmented ensembles, derive pass + model) as one HIP-graph replay per row bucket
    (:mod:`flink_jpmml_amd.runtime.graphs`); 0 = always launch kernel by kernel."""
    device_mirror: bool = False
    """Keep ``[rows]`` device copies of every columnar result (``PredictionBatch.device_out``) next
    to the pinned host scores, so a :class:`~flink_jpmml_amd.parallel.sinks.GatherSink` all-gathers
    them over RCCL without a host round trip (SURVEY §2.6 F5)."""

    # -- dynamic serving
    cache_capacity: int = 64
    """Exact-key LRU capacity of loaded models per operator instance."""
    async_load: bool = True
    """Parse + lower an added model on a background loader thread (the event path only waits if an
    event needs the model before the load finished)."""

    # -- fault tolerance
    checkpoint_dir: Optional[str] = None
    watchdog_s: Optional[float] = None
    """Arm a progress watchdog in the distributed loop: abort the rank when no element was processed
    for this long (a peer stuck in a collective cannot be interrupted from Python)."""

    plan_opts: Dict[str, Any] = field(default_factory=dict)
    """Extra lowering options forwarded to :func:`flink_jpmml_amd.runtime.plans.compile_plan`."""

    def __post_init__(self) -> None:
        if self.precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}, got {self.precision!r}")
        if self.udf_mode not in ("deferred", "replay"):
            raise ValueError(f"udf_mode must be 'deferred' or 'replay', got {self.udf_mode!r}")
        if self.fallback not in FALLBACKS:
            raise ValueError(f"fallback must be one of {FALLBACKS}, got {self.fallback!r}")
        if self.batch_size is not None and int(self.batch_size) < 1:
            raise ValueError("batch_size must be >= 1")
        if self.max_batch_latency_ms is not None and float(self.max_batch_latency_ms) < 0:
            raise ValueError("max_batch_latency_ms must be >= 0")
        if self.micro_batch < 1 or self.pipeline_depth < 1 or self.max_inflight < 1:
            raise ValueError("micro_batch, pipeline_depth and max_inflight must be >= 1")

    # ------------------------------------------------------------------ helpers
    def replace(self, **kw) -> "ScoringConfig":
        return dataclasses.replace(self, **{k: v for k, v in kw.items() if v is not None})

    def lowering_opts(self) -> Dict[str, Any]:
        """Options for ``compile_plan`` implied by the precision policy plus ``plan_opts``."""
        opts = dict(self.plan_opts)
        if self.precision != "fp32":
            opts.setdefault("precision", self.precision)  # mapped per model family by compile_plan
        return opts

    def resolve_device(self, local_rank: int = 0):
        """The device this process scores on (``None`` = host)."""
        if self.device is None:
            return None
        import torch

        if isinstance(self.device, str) and self.device == "auto":
            if not torch.cuda.is_available():
                return None
            dev = torch.device("cuda")
        else:
            dev = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        if dev.type != "cuda":
            return None if dev.type == "cpu" else dev
        if self.device_ids is not None:
            return torch.device("cuda", int(self.device_ids[local_rank % len(self.device_ids)]))
        if dev.index is None:
            n = max(1, torch.cuda.device_count())
            return torch.device("cuda", local_rank % n)
        return dev

    @staticmethod
    def from_env(prefix: str = "FJA_", **overrides) -> "ScoringConfig":
        def get(name, conv):
            v = os.environ.get(prefix + name)
            return conv(v) if v not in (None, "") else None

        kw = dict(batch_size=get("BATCH_SIZE", int), max_batch_latency_ms=get("MAX_BATCH_LATENCY_MS", float),
                  device=get("DEVICE", str), precision=get("PRECISION", str), fallback=get("FALLBACK", str),
                  micro_batch=get("MICRO_BATCH", int), cache_capacity=get("CACHE_CAPACITY", int),
                  checkpoint_dir=get("CHECKPOINT_DIR", str), watchdog_s=get("WATCHDOG_S", float),
                  graph_max_rows=get("GRAPH_MAX_ROWS", int), metrics_port=get("METRICS_PORT", int),
                  host_threads=get("HOST_THREADS", int))
        kw = {k: v for k, v in kw.items() if v is not None}
        kw.update({k: v for k, v in overrides.items() if v is not None})
        return ScoringConfig(**kw)


def merge_config(config: Optional[ScoringConfig], **legacy) -> ScoringConfig:
    """Combine an explicit ``config`` with the legacy keyword arguments of the DSL
    (``batch_size=``, ``device=``, ``plan_opts=``, ``cache_capacity=``): explicit keywords win."""
    base = config if config is not None else ScoringConfig()
    kw = {k: v for k, v in legacy.items() if v is not None}
    if "plan_opts" in kw:
        kw["plan_opts"] = {**base.plan_opts, **kw["plan_opts"]}
    return dataclasses.replace(base, **kw) if kw else base


__all__ = ["FALLBACKS", "PRECISIONS", "ScoringConfig", "merge_config"]
