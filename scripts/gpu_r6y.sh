set -o pipefail
# r6y: final validation — every seed of the randomized GPU files (FJA_FULL_SUITE=1), the per-record
# device rate, smoke, bench N=1.
O=gpurun_out/r6y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
FJA_FULL_SUITE=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --durations=10 -rf > $O/pytest_full.log 2>&1
rc=$?; echo "full suite rc=$rc"; tail -2 $O/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -m pytest tests/test_gpu_per_record.py -m gpu -q -s --timeout 150 --timeout-method thread > $O/per_record.log 2>&1 || { tail -20 $O/per_record.log; exit 1; }
grep "records/s" $O/per_record.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['n_gpus'], d['check'])"
exit $rc
