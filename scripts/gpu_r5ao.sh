set -o pipefail
# r5ao: randomized derived-field expression fuzz: derive kernel vs its numpy twin, column for column
O=gpurun_out/r5ao
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_expr_fuzz.py tests/test_gpu_kernels.py -k "derive or derived or expr" -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
