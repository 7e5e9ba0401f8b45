set -o pipefail
# r6ac: RF votes (one-hot leaf pairs) on LTOP with 8 vs 6 walks per lane.
O=gpurun_out/r6ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model rf --configs auto,ltop6,auto,ltop6,auto,ltop6 > $O/sweep_rf.jsonl 2> $O/sweep_rf.err || { tail -20 $O/sweep_rf.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep_rf.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('rf', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
