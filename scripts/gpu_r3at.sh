set -o pipefail
# binary record source on positional reads (os.preadv into pinned slices): end-to-end bench, 8 / 16 threads.
mkdir -p gpurun_out/r3at
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u -m pytest tests/test_binary_source.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r3at/pytest.log 2>&1 || { tail -30 gpurun_out/r3at/pytest.log; exit 1; }
tail -1 gpurun_out/r3at/pytest.log
for th in 8 16; do
  timeout -k 10 300 python -u bench.py --source binary --steps 5 --warmup 2 --passes 4 --ingest-threads $th > gpurun_out/r3at/bench_binary_t$th.json 2> gpurun_out/r3at/bench_binary_t$th.err || { tail -20 gpurun_out/r3at/bench_binary_t$th.err; exit 1; }
  cut -c1-250 gpurun_out/r3at/bench_binary_t$th.json
done
