#!/bin/bash
# round-2 GPU session K: MLP per-phase timers, bench with calibrated H2D streams, full GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for prec in bf16 fp32; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision $prec --mlp-prof >> gpurun_out/r2k_kbench_mlp.jsonl || exit $?
done
cat gpurun_out/r2k_kbench_mlp.jsonl
for m in gbdt rf; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 >> gpurun_out/r2k_bench.jsonl 2>> gpurun_out/r2k_bench.err || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/r2k_bench.jsonl"):
    d = json.loads(l)
    print(d["config"]["model"][:40], round(d["value"] / 1e6, 1), "M rec/s", d.get("h2d_gbps_effective"), d["config"].get("h2d_streams"))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2k_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2k_pytest_gpu.log | tail -20
exit $rc
