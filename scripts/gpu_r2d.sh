#!/bin/bash
# round-2 GPU session D: new MLP kernel — tests, kernel-only TFLOP/s, rocprof
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -k "mlp or roundtrip" -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d_pytest_mlp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r2d_pytest_mlp.log
if [ $rc -gt 1 ]; then exit $rc; fi
for prec in bf16 fp32; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision $prec >> gpurun_out/r2d_kbench_mlp.jsonl || exit $?
done
cat gpurun_out/r2d_kbench_mlp.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r2d_prof -o mlp -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 10 --precision bf16 > gpurun_out/r2d_rocprof.log 2>&1 || echo "rocprof rc=$?"
find gpurun_out/r2d_prof -name "*stats*" | head
