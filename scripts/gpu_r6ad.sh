set -o pipefail
# r6ad: LTOP with paired deep levels (slots i and i+4 share a gather per step from level 7 / 9).
O=gpurun_out/r6ad
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -m gpu -x -q --timeout 200 --timeout-method thread -k shallow > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,ltop_pair7,ltop_pair9,auto,ltop_pair7,ltop_pair9 > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'], d.get('max_abs_err'))
"
done
