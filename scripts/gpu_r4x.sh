set -o pipefail
# persistent K = 64 first-layer kernel (gemm_k64p_kernel): GPU bit-identity tests, then 1024^3 bf16
# MLP kernel stats, default vs flag 0x200 (one tile per workgroup); input stage with LDS tables
O=gpurun_out/r4x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_wide_mlp.py -m gpu -x -q --timeout 180 --timeout-method thread -rf -k "transposed or k64 or fused_input or wide_gemm_kernels" > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -3 $O/pytest_mlp.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_$n -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_$n.log 2>&1 || return 1
  grep '^{' $O/mlp_$n.log | tail -1
}
run k64p FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0 && run k64 FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0x200 || exit 1
for f in 0 0x200; do
  env FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=$f ITERS=30 timeout -k 10 120 python3 scripts/mlp_prof.py > $O/plain_$f.json 2>&1 || exit 1
  tail -1 $O/plain_$f.json
done
echo done
