#!/usr/bin/env python3
"""Kernel-only micro-benchmark (device-resident records) for profiling the scoring kernels.

python scripts/kbench.py --model gbdt --rows 1048576 --iters 20
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gbdt", choices=["gbdt", "gbdt-binary", "rf", "kmeans", "kmeans-big", "mlp", "svm", "lr", "pcie"])
    p.add_argument("--rows", type=int, default=1 << 20)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--trees", type=int, default=1000)
    p.add_argument("--depth", type=int, default=6)
    p.add_argument("--features", type=int, default=32)
    p.add_argument("--missing", type=float, default=0.0)
    p.add_argument("--layout", default="auto")
    p.add_argument("--lds-budget", type=int, default=80 * 1024)
    p.add_argument("--variant", default="auto")
    p.add_argument("--mlp-prof", action="store_true", help="MLP: per-phase s_memtime ticks of workgroup 0")
    p.add_argument("--clusters", type=int, default=256)
    p.add_argument("--n-sv", type=int, default=256, help="svm: support vectors")
    p.add_argument("--classes", type=int, default=2, help="svm: classes (> 2: one-against-one machines)")
    p.add_argument("--svm-impl", default="auto", choices=["auto", "fused", "wide", "gemm"])
    p.add_argument("--nan-mode", default="auto")
    p.add_argument("--tree-prof", action="store_true", help="tree: per-wave phase ticks of one workgroup")
    p.add_argument("--max-chunk-trees", type=int, default=0)
    p.add_argument("--head-depth", type=int, default=0, help="hybrid layout: PERFECT head levels (4/6/8/10)")
    p.add_argument("--pointer-schedule", default="lockstep", choices=["refill", "lockstep"])
    p.add_argument("--node-order", default="bfs", choices=["bfs", "dfs"])
    p.add_argument("--node-format", default="wide", choices=["auto", "compact", "wide"])
    p.add_argument("--pointer-ilp", type=int, default=8, choices=[2, 4, 8, 16])
    p.add_argument("--p-split", type=float, default=None, help="rf generator: split probability per node (gbdt: fixed 0.9)")
    p.add_argument("--xcd-split", default="off", choices=["on", "off"], help="pointer/hybrid: XCD tree slices")
    p.add_argument("--cache-dir", default="", help="tree models: reuse the generated PMML text across runs")
    p.add_argument("--splits", type=int, default=0, help="tree: force this many tree splits (0 = auto)")
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp8"])
    p.add_argument("--hidden", default="256,256", help="mlp hidden widths")
    p.add_argument("--mlp-kernel", default="auto", choices=["auto", "reg", "panel"], help="bf16 MLP kernel")
    p.add_argument("--mlp-impl", default="auto", choices=["auto", "fused", "wide", "gemm"],
                   help="MLP plan: fused kernel, wide-layer MFMA GEMM, or library GEMM")
    args = p.parse_args()
    import numpy as np
    import torch

    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    if args.model == "pcie":
        F = args.features
        Xh = torch.from_numpy(synth.stream_matrix(args.rows, F, seed=1)).pin_memory()
        Xd = torch.empty_like(Xh, device="cuda")
        res = {}
        for name, fn in (("h2d", lambda: Xd.copy_(Xh, non_blocking=True)), ("d2h", lambda: Xh.copy_(Xd, non_blocking=True))):
            fn(); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.iters
            res[name + "_GBps"] = Xh.numel() * 4 / dt / 1e9
        print(json.dumps({"model": "pcie", "bytes": Xh.numel() * 4, **res}))
        return
    cache = None
    if args.cache_dir and args.model.startswith(("gbdt", "rf")):
        os.makedirs(args.cache_dir, exist_ok=True)
        cache = os.path.join(args.cache_dir, f"{args.model}_{args.trees}_{args.depth}_{args.features}_{args.p_split}.pmml")
    if cache and os.path.exists(cache):
        with open(cache) as fh:
            txt = fh.read()
    elif args.model == "gbdt":
        txt = synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features)
    elif args.model == "gbdt-binary":
        txt = synth.gbdt_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, objective="binary")
    elif args.model == "rf":
        kw = {"p_split": args.p_split} if args.p_split is not None else {}
        txt = synth.random_forest_pmml(n_trees=args.trees, depth=args.depth, n_features=args.features, **kw)
    elif args.model == "mlp":
        txt = synth.mlp_pmml(n_features=args.features, hidden=tuple(int(x) for x in args.hidden.split(",")))
    elif args.model == "svm":
        txt = synth.svm_pmml(n_features=args.features, n_sv=args.n_sv, n_classes=args.classes, gamma=0.05)
    elif args.model == "kmeans-big":
        txt = synth.kmeans_pmml(n_clusters=args.clusters, n_features=args.features, weighted=True)
    elif args.model == "lr":
        txt = synth.iris_logistic_pmml()
    else:
        from flink_jpmml_amd.assets import kmeans_pmml

        txt = kmeans_pmml()
    if cache and not os.path.exists(cache):
        with open(cache, "w") as fh:
            fh.write(txt)
    c = CompiledPmml.from_string(txt)
    opts = {}
    if args.model.startswith(("gbdt", "rf")):
        opts = dict(layout=args.layout, lds_budget=args.lds_budget, variant=args.variant, nan_mode=args.nan_mode,
                    max_chunk_trees=args.max_chunk_trees, head_depth=args.head_depth,
                    pointer_schedule=args.pointer_schedule, node_order=args.node_order,
                    node_format=args.node_format, pointer_ilp=args.pointer_ilp, xcd_split=args.xcd_split,
                    splits=args.splits)
    elif args.model == "kmeans-big":
        opts = dict(cluster_variant=args.variant)
    elif args.model == "svm" and args.svm_impl != "auto":
        opts = dict(svm_impl=args.svm_impl)
    if args.precision != "fp32":
        opts["precision"] = args.precision
    if args.model == "mlp" and args.mlp_impl != "auto":
        opts["mlp_impl"] = args.mlp_impl
    plan = c.plan("cuda:0", **opts)
    if args.model == "mlp" and args.mlp_kernel != "auto" and hasattr(plan, "set_kernel"):
        plan.set_kernel(args.mlp_kernel)
    F = c.n_features
    X = torch.from_numpy(synth.stream_matrix(args.rows, F, seed=1, missing_rate=args.missing)).cuda()
    s = torch.empty(args.rows, device="cuda")
    v = torch.empty(args.rows, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        plan.launch(X, s, v)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        plan.launch(X, s, v)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    prof = None
    if args.model == "mlp" and args.mlp_prof:
        plan.prof = torch.zeros(6, dtype=torch.int64, device="cuda")
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        st, ch, ba, ep, tiles, steps = plan.prof.cpu().tolist()
        if getattr(plan, "reg_kernel", 0):  # register-weight kernel: per-block phases (incl. barrier)
            blocks = max(steps, 1)
            prof = {"ticks_per_block": {"p0": st / blocks, "p1": ch / blocks, "p2": ba / blocks,
                                        "p3": ep / blocks, "p4": tiles / blocks}, "blocks": steps}
        else:
            prof = {"ticks_stage_per_tile": st / max(tiles, 1), "ticks_chain_per_step": ch / max(steps, 1),
                    "ticks_barrier_per_step": ba / max(steps, 1), "ticks_epilogue_per_tile": ep / max(tiles, 1),
                    "tiles": tiles, "steps": steps, "total_ticks": st + ch + ba + ep}
        plan.prof = None
    if args.tree_prof and args.model.startswith(("gbdt", "rf")):
        plan.prof = torch.zeros(64, dtype=torch.int64, device="cuda")
        plan._args = {}
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        w = plan.prof.cpu().view(16, 4).tolist()
        prof = {"per_wave_stage_trav_barrier_total": w,
                "mean": [sum(r[k] for r in w) / 16 for k in range(4)]}
        plan.prof = None
        plan._args = {}
    flops = None
    if args.model == "mlp":
        dims = [F] + [int(x) for x in args.hidden.split(",")] + [1]
        flops = 2.0 * args.rows * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    elif args.model == "svm" and type(plan).__name__ == "SvmWidePlan":  # the MFMA work as issued (padded)
        flops = 2.0 * args.rows * plan.n_tiles * 32 * (plan.fmax + plan.n_groups * plan.mt * 32)
    print(json.dumps({"model": args.model, "rows": args.rows, "features": F, "ms": ms,
                      "tflops": (flops / ms / 1e9) if flops else None, "precision": args.precision,
                      "rows_per_s": args.rows / ms * 1e3, "plan": type(plan).__name__,
                      "layout": getattr(plan, "layout", None), "chunk_trees": getattr(plan, "chunk_trees", None),
                      "head_depth": getattr(plan, "head_depth", None), "depth": getattr(plan, "depth", None),
                      "pointer_schedule": args.pointer_schedule, "node_order": args.node_order, "node_format": args.node_format, "pointer_ilp": args.pointer_ilp,
                      "trees": getattr(plan, "n_trees", None), "xcd_split": getattr(plan, "xcd_split", None),
                      "splits": plan._auto_splits(args.rows) if hasattr(plan, "_auto_splits") else None,
                      "missing": args.missing, "lds_budget": args.lds_budget,
                      "variant": getattr(plan, "variant", None), "mlp_prof": prof,
                      "mlp_kernel": ("reg" if getattr(plan, "reg_kernel", 0) else "panel") if args.model == "mlp" else None}))


if __name__ == "__main__":
    main()
