set -o pipefail
# r6b: default GPU suite (native oracles, trimmed fuzz seeds) with durations, host-path rates on
# the box CPU, bench N=1
O=gpurun_out/r6b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_per_record.py tests/test_field_value_lists.py tests/test_chain_fuzz.py tests/test_mixture_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -rf > $O/pytest_new.log 2>&1 || { tail -60 $O/pytest_new.log; exit 1; }
grep -E "passed|failed|records/s" $O/pytest_new.log | tail -5
timeout -k 10 120 python3 scripts/host_rate.py > $O/host_rate.json 2>&1 || { tail -20 $O/host_rate.json; exit 1; }
cat $O/host_rate.json
timeout -k 10 820 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=60 -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo done
