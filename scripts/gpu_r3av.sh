set -o pipefail
# H2D calibration tie-break toward 2 streams: default bench (auto) vs pinned 1 / 2 copy streams.
mkdir -p gpurun_out/r3av
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py > gpurun_out/r3av/bench_auto.json 2> gpurun_out/r3av/bench_auto.err || { tail -20 gpurun_out/r3av/bench_auto.err; exit 1; }
cut -c1-160 gpurun_out/r3av/bench_auto.json
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --h2d-streams $k > gpurun_out/r3av/bench_h2d$k.json 2> gpurun_out/r3av/bench_h2d$k.err || { tail -20 gpurun_out/r3av/bench_h2d$k.err; exit 1; }
  cut -c1-160 gpurun_out/r3av/bench_h2d$k.json
done
python - <<'PY'
import json
for n in ("auto", "h2d1", "h2d2"):
    d = json.load(open(f"gpurun_out/r3av/bench_{n}.json"))
    print(n, round(d["value"] / 1e6, 1), "M rec/s", "h2d_streams", d.get("config", {}).get("h2d_streams"), "p50", d.get("p50_ms"))
PY
