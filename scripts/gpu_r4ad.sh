set -o pipefail
# next-round input: store-side PMC of the wide-MLP launches (1024^3 bf16, fused head): the
# persistent K = 64 layer and the phase-interleaved layers (kernel trace only, own pass)
O=gpurun_out/r4ad
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
env FUSE_INPUT=0 FUSE_HEAD=1 ITERS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum WRITE_SIZE -d $O/mlp_pmc -o pmc -- python3 scripts/mlp_prof.py > $O/mlp_pmc.log 2>&1 || { tail -20 $O/mlp_pmc.log; exit 1; }
grep '^{' $O/mlp_pmc.log | tail -1
echo done
