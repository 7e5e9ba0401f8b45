set -o pipefail
# r6g: pointer walk without the LDS bad[] array (each thread stages its own row, verdict in a
# register): 32 features x 256 rows = 32 KiB -> 5 workgroups per CU instead of 4. Tests of every
# pointer-walk variant, then the deep-forest sweep (300 trees x depth 14, 1M rows, kernel only).
O=gpurun_out/r6g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py tests/test_inline_leaves.py tests/test_rank3.py tests/test_gpu_tree_fuzz.py tests/test_mixed_models.py tests/test_segmented.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs pointer,pointer+peel,pointer+uskip,pointer,pointer+xcd,pointer16+uskip > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
done
