set -o pipefail
# round 4 validation of HEAD: full GPU suite, smoke(), default bench (headline), --models 64,
# --source text, rocprofv3 kernel stats of the headline bench. A test failure (exit 1) continues;
# a fault / abort / timeout ends the script.
O=gpurun_out/r4m
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
tail -8 $O/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 400 python -u bench.py --models 64 --steps 10 --warmup 2 --passes 8 > $O/bench_models64.json 2> $O/bench_models64.err || { tail -20 $O/bench_models64.err; exit 1; }
tail -c 300 $O/bench_models64.json
timeout -k 10 400 python -u bench.py --source text --steps 4 --warmup 1 --passes 2 --ingest-threads 16 > $O/bench_text.json 2> $O/bench_text.err || { tail -20 $O/bench_text.err; exit 1; }
tail -c 300 $O/bench_text.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 3 --warmup 1 > $O/prof_bench.log 2>&1; rc=$?
tail -2 $O/prof_bench.log; exit $rc
