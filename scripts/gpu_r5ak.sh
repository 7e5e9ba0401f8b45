set -o pipefail
# r5ak: binomial GLM classification (generalizedLinear, mirrored links) through the design lowering
O=gpurun_out/r5ak
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_field_value_lists.py tests/test_nn_field_prep.py tests/test_design.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
