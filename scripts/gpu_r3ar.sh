set -o pipefail
# uniform-skip pointer walk + LDS-head/pointer-tail hybrid: GPU tests, then the deep-forest sweep.
mkdir -p gpurun_out/r3ar
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -x -v --timeout 120 --timeout-method thread -k "uniform_skip or deep_gbdt" > gpurun_out/r3ar/pytest.log 2>&1 || { tail -40 gpurun_out/r3ar/pytest.log; exit 1; }
tail -2 gpurun_out/r3ar/pytest.log
CFG=pointer,hybw2,hybw3,hybw4,hybw6,hybw4u
for m in gbdt rf; do
  timeout -k 10 400 python -u scripts/deep_forest_sweep.py --model $m --configs $CFG >> gpurun_out/r3ar/sweep.jsonl 2>> gpurun_out/r3ar/sweep.err || { tail -20 gpurun_out/r3ar/sweep.err; exit 1; }
done
grep config gpurun_out/r3ar/sweep.jsonl | python -c "import sys,json; [print(d['model'],d['config'],round(d['ms'],3),d['valid_match'],d['max_abs_err']) for d in map(json.loads,sys.stdin)]"
