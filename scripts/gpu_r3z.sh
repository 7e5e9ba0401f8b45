set -o pipefail
# Engine hot-path changes (raw hipMemcpyAsync H2D, one copy stream for small copies, per-thread
# launch structs, wide-kernel split policy): full GPU suite, latency probe, bench.
mkdir -p gpurun_out/r3z
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3z/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3z/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3z/pytest_gpu.log
timeout -k 10 300 python -u scripts/probe_latency.py > gpurun_out/r3z/latency.jsonl 2> gpurun_out/r3z/latency.err || { tail -30 gpurun_out/r3z/latency.err; exit 1; }
cat gpurun_out/r3z/latency.jsonl
timeout -k 10 400 python -u bench.py > gpurun_out/r3z/bench.json 2> gpurun_out/r3z/bench.err || { tail -20 gpurun_out/r3z/bench.err; exit 1; }
cut -c1-200 gpurun_out/r3z/bench.json
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r3z/bench.json").read().strip().splitlines()[-1])
print("value", d["value"] / 1e6, "p50_ms", d["p50_latency_ms"], "p99_ms", d["p99_latency_ms"], "kernel_ms", d["kernel_ms_per_1M_rows"])
PY
