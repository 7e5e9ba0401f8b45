set -o pipefail
# fp32 operands on the wide-layer GEMM (exact-fp32 MFMA): GPU tests, kernel-only vs the library GEMM plan.
mkdir -p gpurun_out/r3aj
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py tests/test_gpu_graphs.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r3aj/pytest.log 2>&1 || { tail -40 gpurun_out/r3aj/pytest.log; exit 1; }
tail -3 gpurun_out/r3aj/pytest.log
for impl in wide gemm; do
  for hid in 1024,1024,512 512 2048,2048; do
    timeout -k 10 200 python -u scripts/kbench.py --model mlp --hidden $hid --features 32 --mlp-impl $impl --precision fp32 >> gpurun_out/r3aj/kbench.jsonl 2>> gpurun_out/r3aj/kbench.err || { tail -20 gpurun_out/r3aj/kbench.err; exit 1; }
  done
done
timeout -k 10 200 python -u scripts/kbench.py --model mlp --hidden 1024,1024,512 --features 32 --mlp-impl wide --precision bf16 >> gpurun_out/r3aj/kbench.jsonl 2>> gpurun_out/r3aj/kbench.err || { tail -20 gpurun_out/r3aj/kbench.err; exit 1; }
cat gpurun_out/r3aj/kbench.jsonl
