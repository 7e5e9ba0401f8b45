set -o pipefail
# r5x: randomized wide-MLP shapes through the persistent kernels
O=gpurun_out/r5x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_wide_mlp.py -m gpu -k "random_shapes" -x -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
