set -o pipefail
mkdir -p gpurun_out/r3ac
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/probe_pull.py > gpurun_out/r3ac/pull.jsonl 2> gpurun_out/r3ac/pull.err || { tail -20 gpurun_out/r3ac/pull.err; exit 1; }
cat gpurun_out/r3ac/pull.jsonl
