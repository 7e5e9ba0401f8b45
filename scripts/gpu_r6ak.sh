set -o pipefail
# r6ak: PMC of the RF (3-class votes) LTOP walk with one-hot leaf pairs vs the clamped walk.
O=gpurun_out/r6ak
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
for C in auto pointer_clamped; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcA_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model rf --configs $C --iters 3 > $O/pmcA_$C.log 2>&1 || { tail -20 $O/pmcA_$C.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmcB_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model rf --configs $C --iters 3 > $O/pmcB_$C.log 2>&1 || { tail -20 $O/pmcB_$C.log; exit 1; }
done
ls $O
