set -o pipefail
# HIP-graph replay for multi-kernel plans: correctness vs eager, latency probe, and the full suite.
mkdir -p gpurun_out/r3af
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3af/pytest_graphs.log 2>&1 || { tail -40 gpurun_out/r3af/pytest_graphs.log; exit 1; }
tail -1 gpurun_out/r3af/pytest_graphs.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3af/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3af/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3af/pytest_gpu.log
