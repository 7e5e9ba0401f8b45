#!/bin/bash
# round-2 GPU session I: full GPU suite; tree kernel with unpadded planes (kbench + PMC); benches
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2i_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2i_pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--features 128" "--model rf" "--model rf --depth 8 --trees 500" "--missing 0.02"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2i_kbench.jsonl || exit $?
done
cut -c1-200 gpurun_out/r2i_kbench.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/r2i_pmc_tree -o tree --output-format csv -- python scripts/kbench.py --iters 3 > gpurun_out/r2i_pmc_tree.log 2>&1 || echo "pmc rc=$?"
for m in gbdt rf; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r2i_bench_$m.json 2> gpurun_out/r2i_bench_$m.err || exit $?
  cut -c1-400 gpurun_out/r2i_bench_$m.json
done
