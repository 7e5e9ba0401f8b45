#!/usr/bin/env python3
"""Small-batch latency breakdown of the headline GBDT (1000 trees, depth 6, 32 features) on one
GPU: kernel only (device-resident rows), H2D + kernel + D2H as plain stream work, the same work
replayed from a captured HIP graph, and the public ``model.predict(RecordBatch)`` path.
Prints one JSON line per batch size."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, q):
    import numpy as np

    return float(np.percentile(xs, q))


def main():
    import numpy as np
    import torch

    from flink_jpmml_amd import PmmlModel
    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix
    from flink_jpmml_amd.config import ScoringConfig
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    kind = os.environ.get("MODEL", "gbdt")
    if kind == "wide_mlp":  # several kernels per launch: input prep + one GEMM per layer + output layer
        from flink_jpmml_amd.bench.synth import mlp_pmml

        txt = mlp_pmml(n_features=32, hidden=(1024, 1024, 512))
        plan_opts = dict(precision="bf16", mlp_impl="wide")
    elif kind == "derived_gbdt":  # derive kernel + tree kernel
        txt = gbdt_pmml(n_trees=500, depth=6, n_features=32, scaled=True)
        plan_opts = {}
    else:
        txt = gbdt_pmml(n_trees=1000, depth=6, n_features=32)
        plan_opts = {}
    c = CompiledPmml.from_string(txt)
    plan = c.plan("cuda:0", **plan_opts)
    model = PmmlModel.from_string(txt).bind(device="cuda:0", config=ScoringConfig(device="cuda:0")) \
        if kind == "gbdt" else None
    iters = int(os.environ.get("ITERS", "200"))
    for n in (256, 1024, 4096, 16384):
        X = stream_matrix(n, c.n_features, seed=3)
        Xh = torch.from_numpy(X).pin_memory()
        Xd = torch.empty_like(Xh, device="cuda")
        s, v = plan.alloc_outputs(n)
        sh = torch.empty(n, dtype=torch.float32).pin_memory()
        vh = torch.empty(n, dtype=torch.uint8).pin_memory()
        st = torch.cuda.Stream()
        res = {"model": kind, "plan": type(plan).__name__, "rows": n,
               "splits": plan._auto_splits(n) if hasattr(plan, "_auto_splits") else None}

        def work():
            Xd.copy_(Xh, non_blocking=True)
            plan.launch(Xd, s, v, stream=st)
            sh.copy_(s, non_blocking=True)
            vh.copy_(v, non_blocking=True)

        # kernel only
        Xd.copy_(Xh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            for _ in range(5):
                plan.launch(Xd, s, v, stream=st)
            e0.record()
            for _ in range(50):
                plan.launch(Xd, s, v, stream=st)
            e1.record()
        torch.cuda.synchronize()
        res["kernel_us"] = e0.elapsed_time(e1) / 50 * 1e3
        # eager stream work, host to host
        lat = []
        with torch.cuda.stream(st):
            for i in range(iters + 10):
                t0 = time.perf_counter()
                work()
                st.synchronize()
                if i >= 10:
                    lat.append((time.perf_counter() - t0) * 1e6)
        res["eager_p50_us"], res["eager_p99_us"] = pct(lat, 50), pct(lat, 99)
        # graph replay of the same work
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(st):
                work()
                st.synchronize()
                with torch.cuda.graph(g, stream=st):
                    work()
            lat = []
            for i in range(iters + 10):
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.current_stream().synchronize()
                st.synchronize()
                if i >= 10:
                    lat.append((time.perf_counter() - t0) * 1e6)
            ref, vref = c.score_matrix_oracle(X)
            tol = 5e-2 if kind == "wide_mlp" else 1e-4  # bf16 operands
            ok = bool((vh.numpy().astype(bool) == vref).all()) and \
                float(np.max(np.abs(sh.numpy()[vref] - ref[vref]) / (1 + np.abs(ref[vref])))) < tol
            res["graph_p50_us"], res["graph_p99_us"], res["graph_correct"] = pct(lat, 50), pct(lat, 99), ok
        except Exception as e:  # noqa: BLE001 - report, keep probing
            res["graph_error"] = f"{type(e).__name__}: {e}"
        # public API
        if model is not None:
            rb = RecordBatch(Xh)
            lat = []
            for i in range(iters + 10):
                t0 = time.perf_counter()
                model.predict(rb).wait()
                if i >= 10:
                    lat.append((time.perf_counter() - t0) * 1e6)
            res["predict_p50_us"], res["predict_p99_us"] = pct(lat, 50), pct(lat, 99)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
