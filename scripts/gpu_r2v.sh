#!/bin/bash
# round-2 GPU session V (re-entry after container restore): full GPU suite + smoke, kernel-only
# numbers for every family, default 1-GPU bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2v_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2v_pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2v_smoke.log 2>&1 || exit $?
cat gpurun_out/r2v_smoke.log
for a in "" "--precision fp8" "--features 128" "--missing 0.02" "--model rf --depth 8 --trees 500" "--model mlp --features 64 --precision bf16" "--model mlp --features 64 --precision fp32" "--model svm" "--model kmeans"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2v_kbench.jsonl || exit $?
done
cut -c1-220 gpurun_out/r2v_kbench.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/r2v_bench.json 2> gpurun_out/r2v_bench.err || exit $?
cut -c1-400 gpurun_out/r2v_bench.json
