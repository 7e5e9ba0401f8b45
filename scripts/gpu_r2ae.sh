#!/bin/bash
# round-2 GPU session AE: full validation of the round's final state — GPU suite, smoke, kernel-only
# table of every family, BASELINE configs 2-5 end to end
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2ae_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2ae_pytest_gpu.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2ae_smoke.log 2>&1 || exit $?
cat gpurun_out/r2ae_smoke.log
for a in "" "--precision fp8" "--features 128" "--missing 0.02" "--model rf --depth 8 --trees 500" "--model mlp --features 64 --precision bf16" "--model mlp --features 64 --precision fp32" "--model svm" "--model kmeans" "--model kmeans-big" "--model lr"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2ae_kbench.jsonl || exit $?
done
python -c "
import json
for l in open('gpurun_out/r2ae_kbench.jsonl'):
    d = json.loads(l); print(d['model'], d['features'], d['precision'], round(d['ms'], 4), 'ms', d.get('tflops'))
"
for m in "--model gbdt" "--model rf" "--model mlp" "--model chain --precision fp8"; do
  timeout -k 10 300 python -u bench.py $m --steps 20 --warmup 3 >> gpurun_out/r2ae_bench.jsonl 2>> gpurun_out/r2ae_bench.err || exit $?
done
python -c "
import json
for l in open('gpurun_out/r2ae_bench.jsonl'):
    d = json.loads(l); print(d['config']['model'][:60], round(d['value'] / 1e6, 1), 'M rec/s', d.get('h2d_gbps_effective'), d.get('kernel_ms_per_1M_rows'), d.get('p50_latency_ms'))
"
echo done
