#!/usr/bin/env python3
"""Interleaved A/B of the phase-interleaved hidden-layer kernels in ONE process (run under
rocprofv3 --kernel-trace; scripts/gemm8p_ab_parse.py reads the trace): HIDDEN layers over ROWS
device-resident rows, each of FLAGS (comma list of GemmArgs flag words) launched ROUNDS times in
turn. Also checks every flag word's scores bit for bit against the first one unless a flag has the
no-store bit (0x2000)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rows = int(os.environ.get("ROWS", 1 << 20))
    hidden = tuple(int(h) for h in os.environ.get("HIDDEN", "1024,1024,4096,1024").split(","))
    flags = [int(f, 0) for f in os.environ.get("FLAGS", "0x1000,0").split(",")]
    rounds = int(os.environ.get("ROUNDS", 3))
    c = CompiledPmml.from_string(mlp_pmml(n_features=32, hidden=hidden, seed=4))
    plan = c.plan("cuda:0", precision="bf16", mlp_impl="wide")
    plan.fuse_input = False
    plan.fuse_head = os.environ.get("FUSE_HEAD", "0") == "1"
    X = torch.from_numpy(stream_matrix(rows, 32, seed=1)).cuda()
    s, v = plan.alloc_outputs(rows)
    ref = None
    same = {}
    for f in flags:  # warm-up + identity
        plan.gemm_flags = f
        plan.launch(X, s, v)
        torch.cuda.synchronize()
        if f & 0x2000:
            continue
        if ref is None:
            ref = (s.clone(), v.clone())
        else:
            same[hex(f)] = bool(torch.equal(ref[1], v) and torch.equal(ref[0][ref[1].bool()], s[v.bool()]))
    for _ in range(rounds):
        for f in flags:
            plan.gemm_flags = f
            plan.launch(X, s, v)
    torch.cuda.synchronize()
    plan.gemm_flags = 0
    print(json.dumps({"hidden": hidden, "rows": rows, "flags": [hex(f) for f in flags], "rounds": rounds,
                      "bit_identical_to_first": same}))


if __name__ == "__main__":
    main()
