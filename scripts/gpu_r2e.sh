#!/bin/bash
# round-2 GPU session E: full GPU suite (wide-kernel modes, new MLP kernel), MLP kernel bench +
# rocprof, bench.py per model family
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r2e_pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for prec in bf16 fp32; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision $prec >> gpurun_out/r2e_kbench_mlp.jsonl || exit $?
done
cat gpurun_out/r2e_kbench_mlp.jsonl
timeout -k 10 120 python -u scripts/kbench.py --model rf --rows 1048576 --iters 20 > gpurun_out/r2e_kbench_rf.jsonl || exit $?
timeout -k 10 120 python -u scripts/kbench.py --model gbdt --features 128 --rows 1048576 --iters 20 >> gpurun_out/r2e_kbench_rf.jsonl || exit $?
cat gpurun_out/r2e_kbench_rf.jsonl
for m in gbdt rf chain mlp; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r2e_bench_$m.json 2> gpurun_out/r2e_bench_$m.err || exit $?
  cat gpurun_out/r2e_bench_$m.json
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e_prof -o mlp -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 10 --precision bf16 > gpurun_out/r2e_rocprof.log 2>&1 || echo "rocprof rc=$?"
find gpurun_out/r2e_prof -name "*stats*"
