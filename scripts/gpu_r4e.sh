set -o pipefail
# round 4: LDS-staged CSV parse kernel + zero-copy registered mapping + two copy streams: GPU text
# tests, ingest probe, --source text bench; rocprofv3 stats of the wide 1024^3 MLP (layer split).
O=gpurun_out/r4e
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_text.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_text.log 2>&1; rc=$?
tail -12 $O/pytest_text.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/text_probe.py > $O/text_probe.json 2> $O/text_probe.err; rc=$?
tail -3 $O/text_probe.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --source text --steps 4 --warmup 1 --passes 2 --ingest-threads 16 > $O/bench_text.json 2> $O/bench_text.err; rc=$?
tail -c 600 $O/bench_text.json; tail -5 $O/bench_text.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ROWS=2097152 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_text -o text -- python3 scripts/text_probe.py > $O/prof_text.log 2>&1; rc=$?
tail -2 $O/prof_text.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python3 scripts/mlp_prof.py > $O/prof_mlp.log 2>&1; rc=$?
tail -2 $O/prof_mlp.log; exit 0
