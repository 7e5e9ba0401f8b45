set -o pipefail
# r5ag: DataField explicit missing-value sentinel (FP_MISSING_VALUE) on every family + prep-heavy suites
O=gpurun_out/r5ag
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_field_value_lists.py tests/test_nn_field_prep.py tests/test_gpu_tree_fuzz.py tests/test_gpu_family_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
