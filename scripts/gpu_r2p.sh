#!/bin/bash
# round-2 GPU session P: reg MLP kernel phase timers
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision bf16 --mlp-kernel reg --mlp-prof >> gpurun_out/r2p_kbench.jsonl || exit $?
cat gpurun_out/r2p_kbench.jsonl
