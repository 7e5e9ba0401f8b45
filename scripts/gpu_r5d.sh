set -o pipefail
# r5d: PMC passes of the LDS-resident deep-forest walk vs the pointer walk (one parse each)
O=gpurun_out/r5d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 scripts/lds_probe.py --configs lds,pointer > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep config $O/trace.log || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o p -- python3 scripts/lds_probe.py --configs lds,pointer --iters 1 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/pmc2 -o p -- python3 scripts/lds_probe.py --configs lds,pointer --iters 1 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
echo done
