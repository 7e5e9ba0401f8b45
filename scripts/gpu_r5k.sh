set -o pipefail
# r5k: per-tile vs per-slice cost of the phase-interleaved hidden layers: K = 1024 vs K = 4096 layers, persistent vs one tile per workgroup
O=gpurun_out/r5k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 0x1000 0; do
  HIDDEN=1024,1024,4096,1024 ITERS=3 FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=$F timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/k_$F -o k -- python3 scripts/mlp_prof.py > $O/k_$F.log 2>&1 || { tail -20 $O/k_$F.log; exit 1; }
  grep hidden $O/k_$F.log || true
done
echo done
