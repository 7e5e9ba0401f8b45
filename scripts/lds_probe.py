#!/usr/bin/env python3
"""Kernel-only timing of the deep-forest layouts on one parsed model (for rocprofv3 PMC passes)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gbdt")
    p.add_argument("--trees", type=int, default=300)
    p.add_argument("--depth", type=int, default=14)
    p.add_argument("--rows", type=int, default=1 << 20)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--configs", default="lds")
    args = p.parse_args()
    import torch

    from flink_jpmml_amd.bench import synth
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    gen = synth.random_forest_pmml if args.model == "rf" else synth.gbdt_pmml
    c = CompiledPmml.from_string(gen(n_trees=args.trees, depth=args.depth, n_features=32, p_split=0.85).encode())
    X = torch.from_numpy(synth.stream_matrix(args.rows, 32, seed=1)).cuda()
    for name in args.configs.split(","):
        kw = dict(layout="pointer", node_format="lds") if name == "lds" else dict(layout="pointer")
        plan = c.plan("cuda:0", **kw)
        s, v = plan.alloc_outputs(args.rows)
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            plan.launch(X, s, v)
        torch.cuda.synchronize()
        print(json.dumps({"config": name, "ms": (time.perf_counter() - t0) / args.iters * 1e3,
                          "chunks": int(plan.lds_chunks.numel() // 4) if plan.lds_chunks is not None else None,
                          "rows_tile": plan.lds_rows, "chunk_u4": plan.lds_chunk_u4}), flush=True)


if __name__ == "__main__":
    main()
