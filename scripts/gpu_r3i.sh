set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_hybrid.py tests/test_gpu_segmented.py tests/test_design.py tests/test_math_context.py tests/test_gpu_surface.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3i/pytest.log 2>&1 || { tail -40 gpurun_out/r3i/pytest.log; exit 1; }
tail -1 gpurun_out/r3i/pytest.log
for M in gbdt rf; do
  for S in lockstep refill; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --pointer-schedule $S --iters 10 >> gpurun_out/r3i/kbench.jsonl 2>> gpurun_out/r3i/kbench.err || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3i/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d["layout"], d.get("pointer_schedule"), round(d["ms"], 3))
PY
