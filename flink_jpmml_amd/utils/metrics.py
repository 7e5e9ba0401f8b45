"""Metrics registry (the reference registers none): counters + latency histograms,
exported as JSON lines or in the Prometheus text exposition format (``prometheus_text``;
``serve_prometheus(port)`` answers ``GET /metrics`` from a daemon thread — per rank, so a
scraper sees each GPU process of a job).

    from flink_jpmml_amd.utils.metrics import METRICS
    METRICS.inc("records_scored", n)
    with METRICS.timer("batch_latency_ms"):
        ...
    METRICS.dump("metrics.jsonl")
"""

from __future__ import annotations

import json
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional

import numpy as np


class Metrics:
    def __init__(self, window: int = 100_000):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = defaultdict(float)
        self.samples: Dict[str, List[float]] = defaultdict(list)
        self.window = window

    def inc(self, name: str, value: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += value

    def observe(self, name: str, value: float) -> None:
        with self._lock:
            s = self.samples[name]
            s.append(value)
            if len(s) > self.window:
                del s[: len(s) - self.window]

    @contextmanager
    def timer(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.observe(name, (time.perf_counter() - t0) * 1e3)

    def summary(self) -> dict:
        with self._lock:
            out = {"counters": dict(self.counters)}
            hist = {}
            for k, v in self.samples.items():
                if v:
                    a = np.asarray(v)
                    hist[k] = {"n": int(a.size), "p50": float(np.percentile(a, 50)), "p99": float(np.percentile(a, 99)),
                               "mean": float(a.mean()), "max": float(a.max())}
            out["histograms"] = hist
            return out

    def dump(self, path: Optional[str] = None) -> str:
        line = json.dumps({"ts": time.time(), **self.summary()})
        if path:
            with open(path, "a") as fh:
                fh.write(line + "\n")
        return line

    def prometheus_text(self, prefix: str = "fja_", labels: Optional[Dict[str, str]] = None) -> str:
        """Counters as ``counter`` samples, latency histograms as ``summary`` quantiles (p50 /
        p99 over the sliding window) + ``_count`` / ``_sum``. Names: dots and dashes become
        underscores under ``prefix``."""
        lab = ""
        if labels:
            lab = "{" + ",".join(f'{k}="{v}"' for k, v in sorted(labels.items())) + "}"

        def name(k: str) -> str:
            return prefix + "".join(c if c.isalnum() else "_" for c in k)

        lines: List[str] = []
        with self._lock:
            counters = dict(self.counters)
            samples = {k: np.asarray(v) for k, v in self.samples.items() if v}
        for k in sorted(counters):
            n = name(k)
            lines += [f"# TYPE {n} counter", f"{n}{lab} {counters[k]:.17g}"]
        for k in sorted(samples):
            a = samples[k]
            n = name(k)
            lines.append(f"# TYPE {n} summary")
            for q in (0.5, 0.99):
                ql = f'quantile="{q}"'
                lq = "{" + (lab[1:-1] + "," if lab else "") + ql + "}"
                lines.append(f"{n}{lq} {float(np.percentile(a, q * 100)):.17g}")
            lines += [f"{n}_count{lab} {a.size}", f"{n}_sum{lab} {float(a.sum()):.17g}"]
        return "\n".join(lines) + "\n"

    def serve_prometheus(self, port: int = 0, host: str = "127.0.0.1", labels: Optional[Dict[str, str]] = None):
        """Serve ``GET /metrics`` on a daemon thread; returns the server (``.server_address``
        has the bound port, ``.shutdown()`` stops it)."""
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        reg = self

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802 - http.server API
                if self.path.split("?")[0] != "/metrics":
                    self.send_error(404)
                    return
                body = reg.prometheus_text(labels=labels).encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *args):  # quiet
                pass

        srv = ThreadingHTTPServer((host, int(port)), Handler)
        threading.Thread(target=srv.serve_forever, name="metrics-http", daemon=True).start()
        return srv

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.samples.clear()


METRICS = Metrics()
