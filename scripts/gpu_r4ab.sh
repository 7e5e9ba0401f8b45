set -o pipefail
# round 4 final validation of HEAD (after the two-buffer GEMM transposed stores): full GPU suite, smoke(), default bench, per-record throughput
# (pipelined flush), kernel stats of the headline bench. A test failure (exit 1) continues.
O=gpurun_out/r4ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
tail -6 $O/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt > $O/per_record.jsonl 2> $O/per_record.err || { tail -20 $O/per_record.err; exit 1; }
cat $O/per_record.jsonl
