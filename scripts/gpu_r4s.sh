set -o pipefail
# round 4: RANK3 with 16-bit conflict-free rank planes staged straight from the rows (17 KiB LDS).
# HBM write ceiling probe.
O=gpurun_out/r4s
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_rank3.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; ok $rc || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model gbdt --configs pointer,rank3,rank3_4,rank3_16 > $O/sweep_gbdt.jsonl 2> $O/sweep_gbdt.err; rc=$?
cut -c1-160 $O/sweep_gbdt.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model rf --configs pointer,rank3 > $O/sweep_rf.jsonl 2> $O/sweep_rf.err; rc=$?
cut -c1-160 $O/sweep_rf.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/write_probe.py > $O/write_probe.json 2>&1; rc=$?
cat $O/write_probe.json; exit $rc
