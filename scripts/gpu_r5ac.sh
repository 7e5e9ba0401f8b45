set -o pipefail
# r5ac: randomized shapes of SVM / k-means / k-NN / segmented models vs the fp64 oracle
O=gpurun_out/r5ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_family_fuzz.py -m gpu -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -80 $O/pytest.log; exit 1; }
tail -40 $O/pytest.log
