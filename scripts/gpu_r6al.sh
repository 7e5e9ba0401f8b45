set -o pipefail
# r6al: LTOP with XCD-aware tree slices (each XCD's L2 holds 1/8 of the forest) vs LTOP unsplit.
O=gpurun_out/r6al
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,pointer+xcd,auto,pointer+xcd > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'], d.get('xcd_split'))
"
done
