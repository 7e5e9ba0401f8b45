set -o pipefail
# r5ax: dump device chain results of fuzz seeds 19 / 37 for CPU-side diagnosis
mkdir -p gpurun_out/chain_diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/chain_diag.py
