set -o pipefail
# Deep forests: exec-masked loads of finished walks vs clamped node-0 loads; TA / TCP counters of
# the clamped, masked and compact kernels.
mkdir -p gpurun_out/r3u
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3u/pytest.log 2>&1 || { tail -40 gpurun_out/r3u/pytest.log; exit 1; }
tail -1 gpurun_out/r3u/pytest.log
timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model rf --configs pointer,pointer+masked,compact > gpurun_out/r3u/sweep_rf.jsonl 2> gpurun_out/r3u/sweep_rf.err || { tail -20 gpurun_out/r3u/sweep_rf.err; exit 1; }
timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model gbdt --configs pointer,pointer+masked,compact > gpurun_out/r3u/sweep_gbdt.jsonl 2> gpurun_out/r3u/sweep_gbdt.err || { tail -20 gpurun_out/r3u/sweep_gbdt.err; exit 1; }
python - <<'PY'
import json
for f in ("rf", "gbdt"):
    for l in open(f"gpurun_out/r3u/sweep_{f}.jsonl"):
        d = json.loads(l)
        if "config" in d:
            print(f, d["config"], round(d["ms"], 3), d["variant"], d["valid_match"], "%.1e" % d["max_abs_err"])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in pointer pointer+masked compact; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r3u/pmc_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs $C --iters 3 > gpurun_out/r3u/pmc_$C.log 2>&1 || { tail -20 gpurun_out/r3u/pmc_$C.log; exit 1; }
done
echo done
