#!/bin/bash
# round-2 GPU session L (re-entry baseline): full GPU suite + smoke, kernel-only numbers for every
# model family, end-to-end bench for BASELINE configs 2-5, tree + MLP PMC passes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2l_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2l_pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2l_smoke.log 2>&1 || exit $?
cat gpurun_out/r2l_smoke.log
for a in "" "--features 128" "--missing 0.02" "--model rf --depth 8 --trees 500" "--model mlp --features 64 --precision bf16" "--model mlp --features 64 --precision fp32" "--model svm" "--model kmeans"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2l_kbench.jsonl || exit $?
done
cut -c1-220 gpurun_out/r2l_kbench.jsonl
for m in "--model gbdt" "--model rf" "--model mlp" "--model chain --precision fp8"; do
  timeout -k 10 300 python -u bench.py $m --steps 20 --warmup 3 >> gpurun_out/r2l_bench.jsonl 2>> gpurun_out/r2l_bench.err || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/r2l_bench.jsonl"):
    d = json.loads(l)
    print(d["config"]["model"][:50], round(d["value"] / 1e6, 1), "M rec/s", d.get("h2d_gbps_effective"), d.get("kernel_ms_per_1M_rows"), d["config"].get("h2d_streams"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r2l_stats -o run --output-format csv -- python scripts/kbench.py --iters 5 > gpurun_out/r2l_stats.log 2>&1 || echo "stats rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r2l_pmc_tree -o tree --output-format csv -- python scripts/kbench.py --iters 3 > gpurun_out/r2l_pmc_tree.log 2>&1 || echo "pmc tree rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r2l_pmc_mlp -o mlp --output-format csv -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 3 --precision bf16 > gpurun_out/r2l_pmc_mlp.log 2>&1 || echo "pmc mlp rc=$?"
echo done
