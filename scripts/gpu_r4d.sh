set -o pipefail
# round 4: device CSV ingest probe (stage timers, host read / H2D rates) + rocprofv3 kernel stats
# of the probe; fused segment-reduction kernel + LocalTransformations GPU tests.
O=gpurun_out/r4d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_segmented.py tests/test_segmented.py tests/test_gpu_text.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_seg.log 2>&1; rc=$?
tail -12 $O/pytest_seg.log; ok $rc || exit $rc
timeout -k 10 600 python -u scripts/text_probe.py > $O/text_probe.json 2> $O/text_probe.err; rc=$?
tail -c 3000 $O/text_probe.json; tail -3 $O/text_probe.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ROWS=2097152 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_text -o text -- python3 scripts/text_probe.py > $O/prof_text.log 2>&1; rc=$?
tail -2 $O/prof_text.log
find $O/prof_text -name "*stats*" | head
exit 0
