set -o pipefail
mkdir -p gpurun_out/r3ae
export HSA_ENABLE_IPC_MODE_LEGACY=0
for M in wide_mlp; do
  MODEL=$M ITERS=100 timeout -k 10 300 python -u scripts/probe_latency.py >> gpurun_out/r3ae/latency.jsonl 2>> gpurun_out/r3ae/latency.err || { tail -30 gpurun_out/r3ae/latency.err; exit 1; }
done
cat gpurun_out/r3ae/latency.jsonl
