set -o pipefail
# r5h: chain expression outputs / string labels, wide (<256,256>) segment reduction, predicate + MLP regressions
O=gpurun_out/r5h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_predicates.py -m gpu -x -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
