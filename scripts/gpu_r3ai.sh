set -o pipefail
# BASELINE configs 3-5 end to end on the round-3 engine (random forest, bf16 MLP, fp8 GBDT chain).
mkdir -p gpurun_out/r3ai
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --model rf --steps 10 --warmup 2 > gpurun_out/r3ai/bench_rf.json 2> gpurun_out/r3ai/bench_rf.err || { tail -20 gpurun_out/r3ai/bench_rf.err; exit 1; }
timeout -k 10 300 python -u bench.py --model mlp --steps 10 --warmup 2 > gpurun_out/r3ai/bench_mlp.json 2> gpurun_out/r3ai/bench_mlp.err || { tail -20 gpurun_out/r3ai/bench_mlp.err; exit 1; }
timeout -k 10 300 python -u bench.py --model chain --precision fp8 --steps 10 --warmup 2 > gpurun_out/r3ai/bench_chain_fp8.json 2> gpurun_out/r3ai/bench_chain_fp8.err || { tail -20 gpurun_out/r3ai/bench_chain_fp8.err; exit 1; }
python - <<'PY'
import json
for f in ("rf", "mlp", "chain_fp8"):
    d = json.loads(open(f"gpurun_out/r3ai/bench_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), "M rec/s  p50", round(d["p50_latency_ms"], 3), "ms  kernel", round(d["kernel_ms_per_1M_rows"], 3), "ms/1M  check", d["check"].get("valid_match"), d["check"].get("max_abs_err_vs_fp64"))
PY
