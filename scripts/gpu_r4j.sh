set -o pipefail
# round 4: wide-MLP fusion A/B (kernel stats per variant: unfused / fused head / + k64 first layer /
# + fused input stage) and PMC counters of the RANK3 vs pointer deep-forest walks.
O=gpurun_out/r4j
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_$n -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_$n.log 2>&1 || return 1
  grep '^{' $O/mlp_$n.log | tail -1
}
run base FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=0x40 && run head FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0x40 && run head_k64 FUSE_INPUT=0 FUSE_HEAD=1 && run head_k64_input FUSE_INPUT=1 FUSE_HEAD=1 || exit 1
for C in pointer rank3; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs $C --iters 3 > $O/pmc_$C.log 2>&1 || { tail -20 $O/pmc_$C.log; exit 1; }
done
echo done
