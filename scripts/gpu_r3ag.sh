set -o pipefail
mkdir -p gpurun_out/r3ag
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u scripts/probe_graph_api.py > gpurun_out/r3ag/graph_api.jsonl 2> gpurun_out/r3ag/graph_api.err || { tail -30 gpurun_out/r3ag/graph_api.err; exit 1; }
cat gpurun_out/r3ag/graph_api.jsonl
