set -o pipefail
# r6w: LTOP with a sched_barrier after the level loads, with / without the null test.
O=gpurun_out/r6w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs auto,ltop_sb,ltop_nnsb,ltop_nn,auto,ltop_sb,ltop_nnsb > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'], d.get('max_abs_err'))
"
done
