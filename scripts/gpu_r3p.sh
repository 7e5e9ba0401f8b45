set -o pipefail
# Session re-entry validation of HEAD: full GPU suite, smoke, 1-GPU bench, rocprofv3 kernel stats,
# per-record + binary-source end to end.
mkdir -p gpurun_out/r3p
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3p/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3p/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3p/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3p/smoke.log 2>&1 || { tail -20 gpurun_out/r3p/smoke.log; exit 1; }
tail -1 gpurun_out/r3p/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3p/bench.json 2> gpurun_out/r3p/bench.err || { tail -20 gpurun_out/r3p/bench.err; exit 1; }
cut -c1-300 gpurun_out/r3p/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p/prof -o bench -- python3 bench.py --steps 3 --warmup 1 --passes 2 --latency-iters 5 > gpurun_out/r3p/prof.log 2>&1 || { tail -20 gpurun_out/r3p/prof.log; exit 1; }
timeout -k 10 200 python -u bench.py --source binary --steps 5 --warmup 2 --passes 4 > gpurun_out/r3p/bench_binary.json 2> gpurun_out/r3p/bench_binary.err || { tail -20 gpurun_out/r3p/bench_binary.err; exit 1; }
cut -c1-300 gpurun_out/r3p/bench_binary.json
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt > gpurun_out/r3p/per_record.jsonl 2> gpurun_out/r3p/per_record.err || { tail -20 gpurun_out/r3p/per_record.err; exit 1; }
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt --api to_batches >> gpurun_out/r3p/per_record.jsonl 2>> gpurun_out/r3p/per_record.err || exit 1
cat gpurun_out/r3p/per_record.jsonl
