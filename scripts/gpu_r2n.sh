#!/bin/bash
# round-2 GPU session N: register-weight bf16 MLP kernel — correctness vs oracle, then kernel-only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -v --timeout 120 --timeout-method thread > gpurun_out/r2n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|Timeout|assert" gpurun_out/r2n_pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
for k in reg panel; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision bf16 --mlp-kernel $k >> gpurun_out/r2n_kbench.jsonl || exit $?
done
timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --hidden 128 --rows 1048576 --iters 20 --precision bf16 >> gpurun_out/r2n_kbench.jsonl || exit $?
cut -c1-250 gpurun_out/r2n_kbench.jsonl
