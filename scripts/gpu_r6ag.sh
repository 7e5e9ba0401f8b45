set -o pipefail
# r6ag: profile of the per-record device predict path.
O=gpurun_out/r6ag
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 scripts/per_record_profile.py > $O/profile.txt 2>&1 || { tail -30 $O/profile.txt; exit 1; }
head -40 $O/profile.txt
