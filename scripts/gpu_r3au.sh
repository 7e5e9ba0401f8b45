set -o pipefail
# final validation of the round: full GPU suite, smoke, 1-GPU bench, rocprofv3 kernel stats of the bench, binary source.
mkdir -p gpurun_out/r3au
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3au/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3au/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3au/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3au/smoke.log 2>&1 || { tail -20 gpurun_out/r3au/smoke.log; exit 1; }
tail -2 gpurun_out/r3au/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3au/bench.json 2> gpurun_out/r3au/bench.err || { tail -20 gpurun_out/r3au/bench.err; exit 1; }
tail -c 600 gpurun_out/r3au/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3au/prof -o bench -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r3au/prof_bench.json 2> gpurun_out/r3au/prof.err || { tail -20 gpurun_out/r3au/prof.err; exit 1; }
find gpurun_out/r3au/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 300 python -u bench.py --source binary --steps 10 --warmup 2 --passes 8 --ingest-threads 16 > gpurun_out/r3au/bench_binary.json 2> gpurun_out/r3au/bench_binary.err || { tail -20 gpurun_out/r3au/bench_binary.err; exit 1; }
cut -c1-200 gpurun_out/r3au/bench_binary.json
