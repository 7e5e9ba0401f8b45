set -o pipefail
# r5aa: headline bench under rocprofv3 kernel stats at HEAD (short run)
O=gpurun_out/r5aa
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 bench.py --steps 4 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json; echo
head -8 $O/k/k_kernel_stats.csv
