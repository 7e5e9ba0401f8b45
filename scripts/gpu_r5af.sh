set -o pipefail
# r5af: PMML Target on regression SVMs (all three SVM plans) + SVM / target suites
O=gpurun_out/r5af
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_target.py tests/test_gpu_svm_lr.py tests/test_svm_wide.py tests/test_svm_gemm.py tests/test_gpu_family_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
