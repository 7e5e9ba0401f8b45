#!/bin/bash
# round-2 GPU session F: MLP kernel diagnostics, new wide-mode / Target tests, full GPU suite (no -x)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_mlp.py > gpurun_out/r2f_diag_mlp.jsonl 2>&1; rc=$?
cat gpurun_out/r2f_diag_mlp.jsonl | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2f_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r2f_pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/kbench.py --model gbdt --features 128 --rows 1048576 --iters 20 > gpurun_out/r2f_kbench.jsonl || exit $?
timeout -k 10 120 python -u scripts/kbench.py --model gbdt --features 256 --rows 1048576 --iters 20 >> gpurun_out/r2f_kbench.jsonl || exit $?
timeout -k 10 120 python -u scripts/kbench.py --model rf --rows 1048576 --iters 20 --depth 8 --trees 500 >> gpurun_out/r2f_kbench.jsonl || exit $?
cat gpurun_out/r2f_kbench.jsonl
