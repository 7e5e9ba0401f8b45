set -o pipefail
# r6q: the per-walk poison flags as one bit mask register: tree-plan GPU tests + sweep.
# GPU tests of every tree-plan family, then auto vs peel vs clamped on the deep forests.
O=gpurun_out/r6q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_hybrid.py tests/test_gpu_kernels.py tests/test_inline_leaves.py tests/test_rank3.py tests/test_gpu_tree_fuzz.py tests/test_mixed_models.py tests/test_segmented.py tests/test_gpu_segmented.py tests/test_mixture_gpu.py tests/test_tree_missing_strategies.py tests/test_gpu_per_record.py tests/test_gpu_lds_forest.py tests/test_chain_fuzz.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,pointer+peel,pointer_clamped,auto,pointer+peel,pointer_clamped > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
done
