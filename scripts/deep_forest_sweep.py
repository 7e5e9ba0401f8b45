#!/usr/bin/env python3
"""Kernel-only sweep of deep-forest tree layouts on ONE parsed model (the 200 MB PMML is
generated and parsed once): device-resident rows, CUDA-event timing of ``plan.launch``.

python scripts/deep_forest_sweep.py --model rf --trees 300 --depth 14 --p-split 0.85
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {
    "pointer": dict(layout="pointer", xcd_split="off"),
    "pointer_clamped": dict(layout="pointer", xcd_split="off", pointer_load="clamped"),
    "pointer_inline": dict(layout="pointer", xcd_split="off", pointer_leaf="inline"),
    "pointer_inline+xcd": dict(layout="pointer", xcd_split="on", pointer_leaf="inline"),
    "pointer+xcd": dict(layout="pointer", xcd_split="on"),
    "pointer+masked": dict(layout="pointer", pointer_load="masked"),
    "super": dict(layout="pointer", node_format="super"),
    "rank3": dict(layout="pointer", node_format="rank3"),
    "rank3_4": dict(layout="pointer", node_format="rank3", pointer_ilp=4),
    "rank3_16": dict(layout="pointer", node_format="rank3", pointer_ilp=16),
    "super+xcd": dict(layout="pointer", node_format="super", xcd_split="on"),
    "super16": dict(layout="pointer", node_format="super", pointer_ilp=16),
    "super4": dict(layout="pointer", node_format="super", pointer_ilp=4),
    "super2": dict(layout="pointer", node_format="super", pointer_ilp=2),
    "pointer2": dict(layout="pointer", pointer_ilp=2),
    "pointer4": dict(layout="pointer", pointer_ilp=4),
    "compact": dict(layout="pointer", node_format="compact", xcd_split="off"),
    "compact+xcd": dict(layout="pointer", node_format="compact", xcd_split="on"),
    "refill+xcd": dict(layout="pointer", pointer_schedule="refill", xcd_split="on"),
    "ilp4+xcd": dict(layout="pointer", pointer_ilp=4, xcd_split="on"),
    "ilp16+xcd": dict(layout="pointer", pointer_ilp=16, xcd_split="on"),
    "hybrid4": dict(layout="hybrid", head_depth=4, xcd_split="off"),
    "hybrid4+xcd": dict(layout="hybrid", head_depth=4, xcd_split="on"),
    "hybrid6+xcd": dict(layout="hybrid", head_depth=6, xcd_split="on"),
    "pointer+uskip": dict(layout="pointer", pointer_load="uskip"),
    "pointer4+uskip": dict(layout="pointer", pointer_load="uskip", pointer_ilp=4),
    "pointer16+uskip": dict(layout="pointer", pointer_load="uskip", pointer_ilp=16),
    "hybw2": dict(layout="hybrid", head_depth=2, hybrid_tail="wide"),
    "hybw3": dict(layout="hybrid", head_depth=3, hybrid_tail="wide"),
    "hybw4": dict(layout="hybrid", head_depth=4, hybrid_tail="wide"),
    "hybw3u": dict(layout="hybrid", head_depth=3, hybrid_tail="wide", pointer_load="uskip"),
    "hybw4u": dict(layout="hybrid", head_depth=4, hybrid_tail="wide", pointer_load="uskip"),
    "pointer+peel": dict(layout="pointer", pointer_load="peel"),
    "pointer+ltop": dict(layout="pointer", pointer_load="ltop"),
    "ltop6": dict(layout="pointer", pointer_load="ltop", pointer_ilp=6),
    "ltop_inline": dict(layout="pointer", pointer_load="ltop", pointer_leaf="inline"),
    "lds": dict(layout="pointer", node_format="lds"),
    "auto": dict(),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="rf", choices=["rf", "gbdt"])
    p.add_argument("--trees", type=int, default=300)
    p.add_argument("--depth", type=int, default=14)
    p.add_argument("--features", type=int, default=32)
    p.add_argument("--p-split", type=float, default=0.85)
    p.add_argument("--rows", type=int, default=1 << 20)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--configs", default=",".join(CONFIGS))
    p.add_argument("--check-rows", type=int, default=4096, help="rows compared with the fp64 oracle per config")
    args = p.parse_args()
    import numpy as np
    import torch

    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    t0 = time.perf_counter()
    gen = synth.random_forest_pmml if args.model == "rf" else synth.gbdt_pmml
    txt = gen(n_trees=args.trees, depth=args.depth, n_features=args.features, p_split=args.p_split)
    c = CompiledPmml.from_string(txt.encode())
    del txt
    print(json.dumps({"event": "loaded", "s": time.perf_counter() - t0}), flush=True)
    Xh = synth.stream_matrix(args.rows, c.n_features, seed=1)
    X = torch.from_numpy(Xh).cuda()
    ref, vref = c.score_matrix_oracle(Xh[: args.check_rows])
    for name in args.configs.split(","):
        plan = c.plan("cuda:0", **CONFIGS[name])
        s, v = plan.alloc_outputs(args.rows)
        for _ in range(2):
            plan.launch(X, s, v)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            plan.launch(X, s, v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        sc = s[: args.check_rows].cpu().numpy()
        vc = v[: args.check_rows].cpu().numpy().astype(bool)
        ok = bool((vc == vref).all())
        err = float(np.max(np.abs(sc[vc] - ref[vc]))) if vc.any() else 0.0
        print(json.dumps({"config": name, "model": args.model, "trees": args.trees, "depth": args.depth,
                          "p_split": args.p_split, "rows": args.rows, "ms": ms, "rows_per_s": args.rows / ms * 1e3,
                          "layout": plan.layout, "variant": plan.variant, "xcd_split": plan.xcd_split,
                          "splits": plan._auto_splits(args.rows), "valid_match": ok, "max_abs_err": err}), flush=True)
        del plan, s, v
        c._plans.clear()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
