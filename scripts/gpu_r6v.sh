set -o pipefail
# r6v: LTOP with the null-on-missing test compiled out (forests without null-on-missing nodes).
O=gpurun_out/r6v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,ltop_nn,auto,ltop_nn > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'], d.get('max_abs_err'))
"
done
