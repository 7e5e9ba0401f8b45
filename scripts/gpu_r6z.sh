set -o pipefail
# r6z: one-hot vote leaves as {class, weight} pairs on the pointer walks: the tree-plan GPU tests,
# then the RF deep forest (auto / peel / clamped all read the pairs).
O=gpurun_out/r6z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_ltop.py tests/test_gpu_hybrid.py tests/test_gpu_kernels.py tests/test_inline_leaves.py tests/test_gpu_tree_fuzz.py tests/test_mixed_models.py tests/test_segmented.py tests/test_gpu_segmented.py tests/test_mixture_gpu.py tests/test_tree_missing_strategies.py tests/test_chain_fuzz.py tests/test_gpu_family_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model rf --configs auto,pointer+peel,pointer_clamped,auto,pointer+peel,pointer_clamped > $O/sweep_rf.jsonl 2> $O/sweep_rf.err || { tail -20 $O/sweep_rf.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep_rf.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('rf', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'], d.get('max_abs_err'))
"
