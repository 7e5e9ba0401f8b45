set -o pipefail
# The N > 1 data path on one GPU: a 1-rank RCCL group (--force-dist) now takes the device-mirror
# all-gather sink exactly as N > 1 does; plain N=1 for comparison.
mkdir -p gpurun_out/r3t
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --force-dist --steps 10 --warmup 3 > gpurun_out/r3t/bench_rccl1.json 2> gpurun_out/r3t/bench_rccl1.err || { echo "rccl1 rc=$?"; tail -20 gpurun_out/r3t/bench_rccl1.err; exit 1; }
cut -c1-200 gpurun_out/r3t/bench_rccl1.json
timeout -k 10 300 python bench.py --force-dist --no-allgather --steps 10 --warmup 3 > gpurun_out/r3t/bench_rccl1_nogather.json 2> gpurun_out/r3t/bench_rccl1_nogather.err || { echo "rccl1ng rc=$?"; tail -20 gpurun_out/r3t/bench_rccl1_nogather.err; exit 1; }
cut -c1-200 gpurun_out/r3t/bench_rccl1_nogather.json
python - <<'PY'
import json
for f in ("bench_rccl1", "bench_rccl1_nogather"):
    d = json.loads(open(f"gpurun_out/r3t/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), d["config"]["allgather_sink"], d["config"]["h2d_streams"], d["timed_region_s"], d["metrics"].get("dist.bytes_gathered"))
PY
