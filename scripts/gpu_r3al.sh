set -o pipefail
# wide-layer GEMM: 4-wave pipelined kernel (two slices in flight across raw barriers) vs the 8-wave
# 2-buffer loop; one process, interleaved rounds, identical outputs asserted.
mkdir -p gpurun_out/r3al
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS=0x10,0x30 timeout -k 10 240 python -u scripts/gemm_ab.py > gpurun_out/r3al/ab_bf16.jsonl 2> gpurun_out/r3al/ab.err || { tail -20 gpurun_out/r3al/ab.err; exit 1; }
HIDDEN=2048,2048 VARIANTS=0x10,0x30 timeout -k 10 240 python -u scripts/gemm_ab.py >> gpurun_out/r3al/ab_bf16.jsonl 2>> gpurun_out/r3al/ab.err || { tail -20 gpurun_out/r3al/ab.err; exit 1; }
PRECISION=fp32 VARIANTS=0x11,0x31 timeout -k 10 300 python -u scripts/gemm_ab.py > gpurun_out/r3al/ab_fp32.jsonl 2>> gpurun_out/r3al/ab.err || { tail -20 gpurun_out/r3al/ab.err; exit 1; }
cat gpurun_out/r3al/ab_bf16.jsonl gpurun_out/r3al/ab_fp32.jsonl
