set -o pipefail
# r6ab: every seed of the randomized GPU files after the one-hot vote leaves and the native vote oracle.
O=gpurun_out/r6ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
FJA_FULL_SUITE=1 timeout -k 10 1080 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --durations=30 -rf > $O/pytest_full.log 2>&1
rc=$?; echo "full suite rc=$rc"; tail -3 $O/pytest_full.log
exit $rc
