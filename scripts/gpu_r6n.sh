set -o pipefail
# r6n: LTOP with 16 walks per lane (GBDT sums), then PMC of the LTOP walk vs the clamped walk.
O=gpurun_out/r6n
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -m gpu -x -q --timeout 200 --timeout-method thread -k "uniform_skip_walks or shallow" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model gbdt --configs auto,ltop16,auto,ltop16 > $O/sweep_gbdt.jsonl 2> $O/sweep_gbdt.err || { tail -20 $O/sweep_gbdt.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep_gbdt.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('gbdt', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
for C in auto pointer_clamped; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcA_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs $C --iters 3 > $O/pmcA_$C.log 2>&1 || { tail -20 $O/pmcA_$C.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmcB_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs $C --iters 3 > $O/pmcB_$C.log 2>&1 || { tail -20 $O/pmcB_$C.log; exit 1; }
done
ls $O
