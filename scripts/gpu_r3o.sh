set -o pipefail
mkdir -p gpurun_out/r3o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3o/pytest.log 2>&1 || { tail -40 gpurun_out/r3o/pytest.log; exit 1; }
tail -1 gpurun_out/r3o/pytest.log
for M in gbdt rf; do
  for I in 4 8 16; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --pointer-ilp $I --iters 10 >> gpurun_out/r3o/kbench.jsonl 2>> gpurun_out/r3o/kbench.err || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3o/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d["layout"], d.get("pointer_ilp"), round(d["ms"], 3))
PY
