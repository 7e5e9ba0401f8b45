"""CPU estimate: distinct 128-byte node lines a 64-row wave touches per lock-step level of the
deep-forest pointer walk (16-byte BFS nodes, `runtime/hybrid.py::pack_trees`), for the stream's
own row order vs rows sorted by a key. The walk is bound by the vector memory pipe's per-line
cost (profiles/r3q, r3w: ~26 distinct lines per gather instruction); a row order that makes a
wave's lanes take similar paths would cut that.

Usage: python scripts/row_order_sim.py [--rows 65536] [--trees 60]
"""
import argparse
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from flink_jpmml_amd.bench.synth import gbdt_pmml, stream_matrix  # noqa: E402
from flink_jpmml_amd.runtime.compiled import CompiledPmml  # noqa: E402
from flink_jpmml_amd.runtime.hybrid import pack_trees  # noqa: E402
from flink_jpmml_amd.runtime.plans import ensemble_spec  # noqa: E402


def walk_codes(nodes, root, X):
    """Per level, the node code each row visits (-1 once finished): list of int64 [n]."""
    n = X.shape[0]
    code = np.full(n, root, dtype=np.int64)
    T = nodes[:, 0].view(np.float32)
    meta = nodes[:, 1].astype(np.int64)
    left = nodes[:, 2].view(np.int32).astype(np.int64)
    right = nodes[:, 3].view(np.int32).astype(np.int64)
    out = []
    while (code >= 0).any():
        out.append(code.copy())
        act = code >= 0
        c = np.where(act, code, 0)
        f = meta[c] & 0xFFFF
        x = X[np.arange(n), f]
        isn = np.isnan(x)
        go_r = (x >= T[c]) | (isn & ((meta[c] >> 31) & 1).astype(bool))
        nxt = np.where(go_r, right[c], left[c])
        code = np.where(act, nxt, -1)
    return out


def lines_per_gather(levels, order):
    """Mean distinct 128-B lines over the 64 lanes of a wave, per level-step with any live lane."""
    tot, cnt = 0, 0
    for codes in levels:
        c = codes[order].reshape(-1, 64)
        live = c >= 0
        lines = np.where(live, c >> 3, -1)  # 8 nodes of 16 B per 128-B line
        s = np.sort(lines, axis=1)
        distinct = (np.diff(s, axis=1) != 0).sum(axis=1) + 1 - (s[:, 0] < 0)
        has = live.any(axis=1)
        tot += distinct[has].sum()
        cnt += has.sum()
    return tot / max(cnt, 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=65536)
    p.add_argument("--trees", type=int, default=60)
    args = p.parse_args()
    c = CompiledPmml.from_string(gbdt_pmml(n_trees=args.trees, depth=14, n_features=32, seed=0, p_split=0.85))
    spec = ensemble_spec(c)
    _, nodes, _, roots, _ = pack_trees(spec.trees, spec.weights, 1, 0, False)
    X = stream_matrix(args.rows, 32, seed=1, missing_rate=0.0).astype(np.float32)
    per_tree = [walk_codes(nodes, int(r), X) for r in roots]
    # split-count per feature (the features most trees test first)
    fcount = np.zeros(32)
    for t in spec.trees:
        f = np.asarray(t.feature)
        np.add.at(fcount, f[f >= 0], 1)
    top = np.argsort(-fcount)
    orders = {"stream": np.arange(args.rows)}
    for k in (1, 2, 3, 4):
        q = np.clip(((X[:, top[:k]] + 4.0) / 8.0 * (1 << (30 // k))).astype(np.int64), 0, (1 << (30 // k)) - 1)
        key = np.zeros(args.rows, dtype=np.int64)
        for b in range(30 // k):  # Morton interleave of the k quantized features
            for j in range(k):
                key |= ((q[:, j] >> (30 // k - 1 - b)) & 1) << (30 - 1 - (b * k + j))
        orders[f"morton_top{k}"] = np.argsort(key, kind="stable")
    # leaf path of tree 0 as the key (rows sharing tree 0's path share its lines)
    orders["tree0_path"] = np.lexsort([lv for lv in per_tree[0][::-1]])
    res = {}
    for name, o in orders.items():
        res[name] = float(np.mean([lines_per_gather(lv, o) for lv in per_tree]))
    print(json.dumps({"rows": args.rows, "trees": args.trees, "mean_distinct_lines_per_gather": res}))


if __name__ == "__main__":
    main()
