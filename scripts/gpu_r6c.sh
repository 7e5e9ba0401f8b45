set -o pipefail
# r6c: fixed new GPU tests (sibling mixtures with numeric labels, per-record contract, near
# sentinel), the per-record device rate (printed), the default GPU suite with durations, bench N=1.
O=gpurun_out/r6c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_per_record.py tests/test_mixture_gpu.py tests/test_scorecard.py tests/test_field_value_lists.py -m gpu -v -s --timeout 200 --timeout-method thread -rf > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "passed|failed|records/s" $O/pytest_new.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 820 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --durations=40 -rf > $O/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['check'])"
timeout -k 10 200 python3 scripts/probe_blaslt.py > $O/blaslt.jsonl 2> $O/blaslt.err || { tail -20 $O/blaslt.err; exit 1; }
cat $O/blaslt.jsonl
