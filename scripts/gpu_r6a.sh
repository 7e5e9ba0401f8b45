set -o pipefail
# r6a: full GPU suite with per-test durations (the "full sweep" log) + the new GPU tests,
# bench --gpus 2 spawning its own ranks (gloo, both on the one GPU), bench --gpus 1 headline
O=gpurun_out/r6a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 280 python -u -m pytest tests/test_mixed_models.py -m gpu -x -v --timeout 120 --timeout-method thread -rf > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
FJA_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --passes 4 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -30 $O/bench_gloo2.err; exit 1; }
tail -c 600 $O/bench_gloo2.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['check'])"
timeout -k 10 820 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=0 -rf > $O/pytest_full.log 2>&1 || { tail -40 $O/pytest_full.log; exit 1; }
tail -3 $O/pytest_full.log
echo done
