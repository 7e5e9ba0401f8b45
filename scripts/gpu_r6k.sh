set -o pipefail
# r6k: LTOP pointer walk (levels 0-4 of each lock-step group's trees staged in LDS, double
# buffered): GPU tests, then ltop vs peel vs clamped, 300 trees x depth 14, 1M rows, kernel only.
O=gpurun_out/r6k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in gbdt rf; do
  timeout -k 10 300 python3 scripts/deep_forest_sweep.py --model $m --configs pointer+peel,pointer+ltop,pointer_clamped,pointer+peel,pointer+ltop,pointer+peel,pointer+ltop > $O/sweep_$m.jsonl 2> $O/sweep_$m.err || { tail -20 $O/sweep_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$O/sweep_$m.jsonl'):
    d = json.loads(l)
    if 'ms' in d: print('$m', d['config'], round(d['ms'], 3), d['valid_match'], d['variant'])
"
done
