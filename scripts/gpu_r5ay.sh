set -o pipefail
# r5ay: nullPrediction padding fix (padded PERFECT nodes read the parent split's column): chain fuzz,
# tree fuzz, tree-kernel GPU tests
O=gpurun_out/r5ay
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_chain_fuzz.py tests/test_gpu_tree_fuzz.py tests/test_gpu_kernels.py tests/test_gpu_segmented.py tests/test_gpu_family_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
