set -o pipefail
# XCD-aware tree slices for deep forests: GPU tests, kernel-only sweep, L2 / L1 counters on vs off.
mkdir -p gpurun_out/r3q
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3q/pytest.log 2>&1 || { tail -40 gpurun_out/r3q/pytest.log; exit 1; }
tail -1 gpurun_out/r3q/pytest.log
timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model rf > gpurun_out/r3q/sweep_rf.jsonl 2> gpurun_out/r3q/sweep_rf.err || { tail -20 gpurun_out/r3q/sweep_rf.err; exit 1; }
timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model gbdt --p-split 0.85 > gpurun_out/r3q/sweep_gbdt.jsonl 2> gpurun_out/r3q/sweep_gbdt.err || { tail -20 gpurun_out/r3q/sweep_gbdt.err; exit 1; }
python - <<'PY'
import json
for f in ("rf", "gbdt"):
    for l in open(f"gpurun_out/r3q/sweep_{f}.jsonl"):
        d = json.loads(l)
        if "config" in d:
            print(f, d["config"], round(d["ms"], 3), d["layout"], d["splits"], d["valid_match"], "%.1e" % d["max_abs_err"])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocprofv3 -L > gpurun_out/r3q/counters.txt 2>&1 || true
for C in pointer pointer+xcd; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/r3q/pmc_$C -o pmc -- python3 scripts/deep_forest_sweep.py --model rf --configs $C --iters 3 > gpurun_out/r3q/pmc_$C.log 2>&1 || { tail -20 gpurun_out/r3q/pmc_$C.log; exit 1; }
done
ls -R gpurun_out/r3q | head -40
