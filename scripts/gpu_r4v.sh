set -o pipefail
# transposed-accumulator hidden-layer stores (store_hidden_t): GPU tests, then the 1024^3 bf16 MLP
# kernel stats with the old direct stores (flag 0x100) vs the new default, fused head on / off,
# fused input stage on / off.
O=gpurun_out/r4v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_wide_mlp.py -m gpu -x -q --timeout 180 --timeout-method thread -rf > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -3 $O/pytest_mlp.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_$n -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_$n.log 2>&1 || return 1
  grep '^{' $O/mlp_$n.log | tail -1
}
run old_head FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0x100 && run new_head FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0 && \
run old_nohead FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=0x100 && run new_nohead FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=0 && \
run new_head_input FUSE_INPUT=1 FUSE_HEAD=1 GEMM_FLAGS=0 || exit 1
for n in old_head new_head; do
  env FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=$([ $n = old_head ] && echo 0x100 || echo 0) ITERS=30 timeout -k 10 120 python3 scripts/mlp_prof.py > $O/plain_$n.json 2>&1 || exit 1
  tail -1 $O/plain_$n.json
done
echo done
