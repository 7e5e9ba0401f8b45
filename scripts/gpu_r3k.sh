set -o pipefail
mkdir -p gpurun_out/r3k
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3k/pytest.log 2>&1 || { tail -40 gpurun_out/r3k/pytest.log; exit 1; }
tail -1 gpurun_out/r3k/pytest.log
for M in gbdt rf; do
  for O in dfs bfs; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --node-order $O --iters 10 >> gpurun_out/r3k/kbench.jsonl 2>> gpurun_out/r3k/kbench.err || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3k/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d["layout"], d.get("pointer_schedule"), d.get("node_order"), round(d["ms"], 3))
PY
