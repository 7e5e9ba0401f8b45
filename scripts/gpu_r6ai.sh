set -o pipefail
# r6ai: per-record device predict vs tree slices of the 1-row launch.
O=gpurun_out/r6ai
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 scripts/per_record_splits.py > $O/splits.jsonl 2> $O/splits.err || { tail -30 $O/splits.err; exit 1; }
cat $O/splits.jsonl
