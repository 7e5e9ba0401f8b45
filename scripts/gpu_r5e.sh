set -o pipefail
# r5e: LDS-resident walk with per-lane refill queues: parity + kernel time + PMC (VALU / LDS)
O=gpurun_out/r5e
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_lds_forest.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/lds_probe.py --configs lds,pointer > $O/probe_gbdt.jsonl 2>&1 || { tail -20 $O/probe_gbdt.jsonl; exit 1; }
grep config $O/probe_gbdt.jsonl
timeout -k 10 300 python -u scripts/lds_probe.py --model rf --configs lds,pointer > $O/probe_rf.jsonl 2>&1 || { tail -20 $O/probe_rf.jsonl; exit 1; }
grep config $O/probe_rf.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o p -- python3 scripts/lds_probe.py --configs lds --iters 1 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
echo done
