set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3g/pytest_hybrid.log 2>&1 || { tail -30 gpurun_out/r3g/pytest_hybrid.log; exit 1; }
tail -1 gpurun_out/r3g/pytest_hybrid.log
for M in gbdt rf; do
  for H in 4 6 8; do for C in 8 16 32; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout hybrid --head-depth $H --max-chunk-trees $C --iters 10 >> gpurun_out/r3g/kbench.jsonl 2>> gpurun_out/r3g/kbench.err || exit 1
  done; done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3g/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d["layout"], d["head_depth"], d["chunk_trees"], round(d["ms"], 3))
PY
