set -o pipefail
# r6u: LTOP shape matrix (features, class slots, partial groups, unaligned rows) vs the clamped walk
# and the oracle.
O=gpurun_out/r6u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_ltop.py -m gpu -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -12 $O/pytest.log; exit $rc
