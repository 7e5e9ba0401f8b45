set -o pipefail
# wide-layer GEMM: phase-interleaved bf16 kernel (gemm8_kernel, flag 0x80) vs the 2-buffer loop;
# one process, interleaved rounds, bit-identical outputs asserted. Small shape first.
mkdir -p gpurun_out/r3an
export HSA_ENABLE_IPC_MODE_LEGACY=0
HIDDEN=512 ROWS=65536 VARIANTS=0,0x80 timeout -k 10 120 python -u scripts/gemm_ab.py > gpurun_out/r3an/ab.jsonl 2> gpurun_out/r3an/ab.err || { tail -20 gpurun_out/r3an/ab.err; exit 1; }
VARIANTS=0,0x80 timeout -k 10 120 python -u scripts/gemm_ab.py >> gpurun_out/r3an/ab.jsonl 2>> gpurun_out/r3an/ab.err || { tail -20 gpurun_out/r3an/ab.err; exit 1; }
HIDDEN=2048,2048 VARIANTS=0,0x80 timeout -k 10 120 python -u scripts/gemm_ab.py >> gpurun_out/r3an/ab.jsonl 2>> gpurun_out/r3an/ab.err || { tail -20 gpurun_out/r3an/ab.err; exit 1; }
HIDDEN=512 VARIANTS=0,0x80 timeout -k 10 120 python -u scripts/gemm_ab.py >> gpurun_out/r3an/ab.jsonl 2>> gpurun_out/r3an/ab.err || { tail -20 gpurun_out/r3an/ab.err; exit 1; }
cat gpurun_out/r3an/ab.jsonl
