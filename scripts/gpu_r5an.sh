set -o pipefail
# r5an: randomized MiningField / DataField treatment fuzz on the device (40 random documents)
O=gpurun_out/r5an
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_prep_fuzz.py tests/test_field_value_lists.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
