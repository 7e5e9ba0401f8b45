set -o pipefail
# r6ah: per-record device predict with the prepared row launcher: GPU tests (rates, contract,
# threads, direct sinks) and the profile.
O=gpurun_out/r6ah
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_per_record.py tests/test_gpu_kernels.py tests/test_mixed_models.py tests/test_columnar.py -m gpu -q -s --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "records/s|passed|failed" $O/pytest.log | tail -4
timeout -k 10 300 python3 scripts/per_record_profile.py > $O/profile.txt 2>&1 || { tail -30 $O/profile.txt; exit 1; }
head -24 $O/profile.txt
