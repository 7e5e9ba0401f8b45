set -o pipefail
# round 4: device CSV parse tests, regrouped mixed-model tests, --models 64 bench (own slice ring +
# batched tree launches), --source text bench (device parse), rocprofv3 stats of the models run.
O=gpurun_out/r4c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_text.py tests/test_mixed_models.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?
tail -15 $O/pytest_new.log; ok $rc || exit $rc
timeout -k 10 600 python -u bench.py --models 64 --steps 10 --warmup 2 --passes 8 > $O/bench_models64.json 2> $O/bench_models64.err; rc=$?
tail -c 300 $O/bench_models64.json; tail -3 $O/bench_models64.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --source text --steps 4 --warmup 1 --passes 2 --ingest-threads 16 > $O/bench_text.json 2> $O/bench_text.err; rc=$?
tail -c 600 $O/bench_text.json; tail -5 $O/bench_text.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_models -o models -- python3 bench.py --models 64 --steps 3 --warmup 1 --passes 2 > $O/prof_models.log 2>&1; rc=$?
tail -3 $O/prof_models.log; exit 0
