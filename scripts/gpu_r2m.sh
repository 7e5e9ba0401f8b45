#!/bin/bash
# round-2 GPU session M: MLP per-phase timers (bf16 / fp32), chain fp8 kernel-only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for prec in bf16 fp32; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision $prec --mlp-prof >> gpurun_out/r2m_kbench.jsonl || exit $?
done
for a in "--model gbdt-binary --precision fp8" "--model gbdt-binary" "--model gbdt --precision fp8"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2m_kbench.jsonl || exit $?
done
cat gpurun_out/r2m_kbench.jsonl
