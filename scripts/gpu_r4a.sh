set -o pipefail
# round 4 first validation (fail-closed scanner, sink changes, knn): full GPU suite, smoke, 1-GPU bench.
mkdir -p gpurun_out/r4a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r4a/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4a/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { tail -20 gpurun_out/r4a/smoke.log; exit 1; }
tail -2 gpurun_out/r4a/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || { tail -20 gpurun_out/r4a/bench.err; exit 1; }
tail -c 600 gpurun_out/r4a/bench.json
