set -o pipefail
# r6o: LTOP + inline leaf payloads (no leaf gather) vs LTOP: GPU tests, then the deep forests.
O=gpurun_out/r6o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_inline_leaves.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,ltop_inline,auto,ltop_inline > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
done
