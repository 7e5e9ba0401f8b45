set -o pipefail
mkdir -p gpurun_out/r3h
:
:
for M in gbdt rf; do
  timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --iters 10 >> gpurun_out/r3h/kbench.jsonl 2>> gpurun_out/r3h/kbench.err || exit 1
  for H in 4 6 8; do for C in 8 16 32; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout hybrid --head-depth $H --max-chunk-trees $C --iters 10 >> gpurun_out/r3h/kbench.jsonl 2>> gpurun_out/r3h/kbench.err || exit 1
  done; done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3h/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d["layout"], d.get("head_depth"), d.get("chunk_trees"), round(d["ms"], 3))
PY
