set -o pipefail
# Checkpoint validation: full GPU suite, smoke, 1-GPU bench.
mkdir -p gpurun_out/r3ad
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3ad/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3ad/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3ad/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ad/smoke.log 2>&1 || { tail -20 gpurun_out/r3ad/smoke.log; exit 1; }
tail -1 gpurun_out/r3ad/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3ad/bench.json 2> gpurun_out/r3ad/bench.err || { tail -20 gpurun_out/r3ad/bench.err; exit 1; }
cut -c1-200 gpurun_out/r3ad/bench.json
