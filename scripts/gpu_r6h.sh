set -o pipefail
# r6h: interleaved A/B of the lock-step pointer walk vs PEEL (top two levels from wave-uniform
# scalar loads) on the 32 KiB-LDS pointer kernels, 300 trees x depth 14, 1M rows, kernel only.
O=gpurun_out/r6h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs pointer,pointer+peel,pointer,pointer+peel,pointer,pointer+peel,auto > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
done
