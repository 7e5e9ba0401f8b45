set -o pipefail
# r6aj: final validation after the prepared row launch: host rates, default GPU suite, smoke, bench N=1.
O=gpurun_out/r6aj
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 scripts/host_rate.py > $O/host_rate.json 2> $O/host_rate.err || { tail -20 $O/host_rate.err; exit 1; }
cat $O/host_rate.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --durations=10 -rf > $O/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['n_gpus'], d['check'])"
exit $rc
