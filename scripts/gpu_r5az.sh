set -o pipefail
# r5az: final validation of HEAD after the chain-fuzz fixes, part 1: the full GPU suite
O=gpurun_out/r5az
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -rf --durations=20 -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -30 $O/pytest.log
