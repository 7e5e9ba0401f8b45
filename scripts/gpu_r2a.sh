#!/bin/bash
# round-2 GPU session A: GPU tests + DSL bench + engine bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r2a_pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r2a_bench_dsl.json 2> gpurun_out/r2a_bench_dsl.err || exit $?
cat gpurun_out/r2a_bench_dsl.json
timeout -k 10 300 python -u bench.py --api engine > gpurun_out/r2a_bench_engine.json 2> gpurun_out/r2a_bench_engine.err || exit $?
cat gpurun_out/r2a_bench_engine.json
