set -o pipefail
# wide-layer GEMM: third LDS buffer for the streamed activations (A two slices ahead, counted vmcnt,
# raw barriers) vs the 2-buffer loop; one process, interleaved rounds, identical outputs asserted.
mkdir -p gpurun_out/r3am
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS=0,0x40 timeout -k 10 240 python -u scripts/gemm_ab.py > gpurun_out/r3am/ab.jsonl 2> gpurun_out/r3am/ab.err || { tail -20 gpurun_out/r3am/ab.err; exit 1; }
HIDDEN=2048,2048 VARIANTS=0,0x40 timeout -k 10 240 python -u scripts/gemm_ab.py >> gpurun_out/r3am/ab.jsonl 2>> gpurun_out/r3am/ab.err || { tail -20 gpurun_out/r3am/ab.err; exit 1; }
HIDDEN=512 VARIANTS=0,0x40 timeout -k 10 240 python -u scripts/gemm_ab.py >> gpurun_out/r3am/ab.jsonl 2>> gpurun_out/r3am/ab.err || { tail -20 gpurun_out/r3am/ab.err; exit 1; }
PRECISION=fp32 VARIANTS=0,0x40 timeout -k 10 300 python -u scripts/gemm_ab.py >> gpurun_out/r3am/ab.jsonl 2>> gpurun_out/r3am/ab.err || { tail -20 gpurun_out/r3am/ab.err; exit 1; }
cat gpurun_out/r3am/ab.jsonl
