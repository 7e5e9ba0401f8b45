set -o pipefail
# round 4: new GPU tests (mixed-model grouped pass, no-sync gather, knn exact matches), full GPU
# suite, --models 64 bench, headline bench. A test failure (exit 1) continues; a fault / abort /
# timeout ends the script.
O=gpurun_out/r4b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_mixed_models.py tests/test_gpu_dsl.py tests/test_knn.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?
tail -5 $O/pytest_new.log; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 600 python -u bench.py --models 64 --steps 5 --warmup 2 --passes 4 > $O/bench_models64.json 2> $O/bench_models64.err; rc=$?
tail -c 1500 $O/bench_models64.json; tail -5 $O/bench_models64.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
