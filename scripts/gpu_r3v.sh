set -o pipefail
# Deep forests: SUPER layout (two levels per 16-byte slot) vs the pointer walk; TA counters.
mkdir -p gpurun_out/r3v
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3v/pytest.log 2>&1 || { tail -40 gpurun_out/r3v/pytest.log; exit 1; }
tail -1 gpurun_out/r3v/pytest.log
for M in rf gbdt; do
  timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model $M --configs pointer,super,super+xcd > gpurun_out/r3v/sweep_$M.jsonl 2> gpurun_out/r3v/sweep_$M.err || { tail -20 gpurun_out/r3v/sweep_$M.err; exit 1; }
done
python - <<'PY'
import json
for f in ("rf", "gbdt"):
    for l in open(f"gpurun_out/r3v/sweep_{f}.jsonl"):
        d = json.loads(l)
        if "config" in d:
            print(f, d["config"], round(d["ms"], 3), d["variant"], d["valid_match"], "%.1e" % d["max_abs_err"])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/r3v/pmc_super -o pmc -- python3 scripts/deep_forest_sweep.py --model gbdt --configs super --iters 3 > gpurun_out/r3v/pmc_super.log 2>&1 || { tail -20 gpurun_out/r3v/pmc_super.log; exit 1; }
echo done
