set -o pipefail
# r5w: every BASELINE config and bench mode end to end at HEAD (configs 3-5, --models 64, --source binary / text)
O=gpurun_out/r5w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --model rf --steps 10 --warmup 2 > $O/bench_rf.json 2> $O/bench_rf.err || { tail -20 $O/bench_rf.err; exit 1; }
timeout -k 10 300 python -u bench.py --model mlp --steps 10 --warmup 2 > $O/bench_mlp.json 2> $O/bench_mlp.err || { tail -20 $O/bench_mlp.err; exit 1; }
timeout -k 10 300 python -u bench.py --model chain --precision fp8 --steps 10 --warmup 2 > $O/bench_chain_fp8.json 2> $O/bench_chain_fp8.err || { tail -20 $O/bench_chain_fp8.err; exit 1; }
timeout -k 10 400 python -u bench.py --models 64 --steps 8 --warmup 2 > $O/bench_models64.json 2> $O/bench_models64.err || { tail -20 $O/bench_models64.err; exit 1; }
timeout -k 10 400 python -u bench.py --source binary --steps 8 --warmup 2 > $O/bench_binary.json 2> $O/bench_binary.err || { tail -20 $O/bench_binary.err; exit 1; }
timeout -k 10 400 python -u bench.py --source text --steps 6 --warmup 2 > $O/bench_text.json 2> $O/bench_text.err || { tail -20 $O/bench_text.err; exit 1; }
python - <<'PY'
import json
for f in ("rf", "mlp", "chain_fp8", "models64", "binary", "text"):
    d = json.loads(open(f"gpurun_out/r5w/bench_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), "M rec/s  p50", round(d.get("p50_latency_ms") or -1, 3), "ms  kernel", round(d.get("kernel_ms_per_1M_rows") or -1, 3), "ms/1M  check", d["check"].get("valid_match"), d["check"].get("max_abs_err_vs_fp64"))
PY
