set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_hybrid.py tests/test_wide_mlp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3n/pytest.log 2>&1 || { tail -40 gpurun_out/r3n/pytest.log; exit 1; }
tail -1 gpurun_out/r3n/pytest.log
for M in gbdt rf; do
  for F in wide compact; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --node-format $F --iters 10 >> gpurun_out/r3n/kbench.jsonl 2>> gpurun_out/r3n/kbench.err || exit 1
  done
done
timeout -k 10 180 python -u scripts/kbench.py --model mlp --features 64 --hidden 1024,1024 --precision bf16 --mlp-impl wide --rows 1048576 --iters 10 >> gpurun_out/r3n/kbench.jsonl 2>> gpurun_out/r3n/kbench.err || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r3n/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d.get("plan"), d["layout"], d.get("node_format"), round(d["ms"], 3), d.get("tflops"))
PY
