set -o pipefail
# r5t: where else the persistent phase kernel pays: K = 4096 (bit 16 forces it) and K = 256..448 layers (bit 7 forces the phase path)
O=gpurun_out/r5t
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=1024,1024,4096,1024 FLAGS=0x1000,0x10000,0x12000 ROUNDS=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/k4096 -o k -- python3 scripts/gemm8p_ab.py > $O/k4096.log 2>&1 || { tail -20 $O/k4096.log; exit 1; }
grep hidden $O/k4096.log
python3 scripts/gemm8p_ab_parse.py $O/k4096/k_kernel_trace.csv 3 > $O/k4096_summary.json
HIDDEN=256,256,448,320,512 FLAGS=0,0x80 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/small -o k -- python3 scripts/gemm8p_ab.py > $O/small.log 2>&1 || { tail -20 $O/small.log; exit 1; }
grep hidden $O/small.log
echo done
