set -o pipefail
# Small-batch latency breakdown: kernel only / eager H2D+kernel+D2H / HIP-graph replay / predict();
# text-source ingest after the single-pass parser.
mkdir -p gpurun_out/r3x
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/probe_latency.py > gpurun_out/r3x/latency.jsonl 2> gpurun_out/r3x/latency.err || { tail -30 gpurun_out/r3x/latency.err; exit 1; }
cat gpurun_out/r3x/latency.jsonl
timeout -k 10 400 python -u bench.py --source text --rows 2097152 --steps 3 --warmup 1 --passes 2 --ingest-threads 16 > gpurun_out/r3x/bench_text.json 2> gpurun_out/r3x/bench_text.err || { tail -20 gpurun_out/r3x/bench_text.err; exit 1; }
cut -c1-250 gpurun_out/r3x/bench_text.json
timeout -k 10 300 python -u scripts/ingest_bench.py 1048576 > gpurun_out/r3x/ingest.json 2> gpurun_out/r3x/ingest.err || { tail -20 gpurun_out/r3x/ingest.err; exit 1; }
cat gpurun_out/r3x/ingest.json
