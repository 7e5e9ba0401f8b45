set -o pipefail
# r5m: gemm8p variant ablation (early A1 / asm epilogue / no stores) vs gemm8_kernel, one process, interleaved
O=gpurun_out/r5m
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FLAGS=0x1000,0,0x2000,0x4000,0x6000,0x8000 ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab -o k -- python3 scripts/gemm8p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep hidden $O/ab.log
python3 scripts/gemm8p_ab_parse.py $O/ab/k_kernel_trace.csv > $O/ab_summary.json && cat $O/ab_summary.json
