set -o pipefail
# r5ab: randomized tree ensembles on the automatic plan choice vs the fp64 oracle
O=gpurun_out/r5ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree_fuzz.py -m gpu -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -22 $O/pytest.log
