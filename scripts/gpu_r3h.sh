set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 400 python -u -m pytest tests/test_knn.py tests/test_gpu_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h/pytest_knn_hybrid.log 2>&1 || { tail -40 gpurun_out/r3h/pytest_knn_hybrid.log; exit 1; }
tail -1 gpurun_out/r3h/pytest_knn_hybrid.log
bash scripts/gpu_r3g.sh
