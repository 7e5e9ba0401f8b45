set -o pipefail
# r6af: LTOP shape matrix + tree splits (XCD slices, grid.y splits) vs the clamped walk and the oracle.
O=gpurun_out/r6af
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_ltop.py -m gpu -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -12 $O/pytest.log; exit $rc
