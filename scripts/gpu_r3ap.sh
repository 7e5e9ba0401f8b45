set -o pipefail
# validation after the fp32 wide GEMM + phase-interleaved bf16 GEMM: full GPU suite, smoke, 1-GPU bench,
# kernel-only wide MLP table (bf16 + fp32).
mkdir -p gpurun_out/r3ap
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3ap/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3ap/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3ap/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ap/smoke.log 2>&1 || { tail -20 gpurun_out/r3ap/smoke.log; exit 1; }
tail -2 gpurun_out/r3ap/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3ap/bench.json 2> gpurun_out/r3ap/bench.err || { tail -20 gpurun_out/r3ap/bench.err; exit 1; }
tail -c 600 gpurun_out/r3ap/bench.json
for hid in 1024,1024,512 2048,2048; do
  for prec in bf16 fp32; do
    HIDDEN=$hid PRECISION=$prec ROUNDS=3 timeout -k 10 200 python -u scripts/gemm_ab.py >> gpurun_out/r3ap/wide_mlp.jsonl 2>> gpurun_out/r3ap/wide_mlp.err || { tail -20 gpurun_out/r3ap/wide_mlp.err; exit 1; }
  done
done
cat gpurun_out/r3ap/wide_mlp.jsonl
