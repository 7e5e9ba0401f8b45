set -o pipefail
# round 4: PMC counters of the RANK3 walk vs the 16-byte pointer walk (300 trees x depth 14 GBDT):
# TA / TCP line accesses, VMEM and LDS instructions (VERDICT r3 item 3 asks for
# TCP_TOTAL_CACHE_ACCESSES_sum and SQ_INSTS_LDS).
O=gpurun_out/r4i
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in pointer rank3; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs $C --iters 3 > $O/pmc_$C.log 2>&1 || { tail -20 $O/pmc_$C.log; exit 1; }
done
echo done
