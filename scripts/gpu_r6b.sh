set -o pipefail
# r6b: new GPU tests (per-record device path, value lists, chain fuzz explanations, sibling
# mixtures), host-path rates on the box CPU, then the default GPU suite with durations.
# A plain test failure (rc 1) does not stop the script; a timeout / abort / crash does.
O=gpurun_out/r6b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_per_record.py tests/test_field_value_lists.py tests/test_chain_fuzz.py tests/test_mixture_gpu.py tests/test_scorecard.py -m gpu -v --timeout 200 --timeout-method thread -rf > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "passed|failed|records/s" $O/pytest_new.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python3 scripts/host_rate.py > $O/host_rate.json 2>&1 || { tail -20 $O/host_rate.json; exit 1; }
cat $O/host_rate.json
timeout -k 10 820 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --durations=60 -rf > $O/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/pytest.log
exit $rc
