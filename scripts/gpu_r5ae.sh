set -o pipefail
# r5ae: NeuralNetworks with MiningField / DataField treatments behind a prepare pass (was: treatment silently skipped)
O=gpurun_out/r5ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_nn_field_prep.py tests/test_gpu_mlp.py tests/test_wide_mlp.py tests/test_gpu_graphs.py tests/test_gpu_segmented.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
