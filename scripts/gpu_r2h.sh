#!/bin/bash
# round-2 GPU session G: MLP glds panel pipeline (correctness + speed), full GPU suite, tree PMC
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_mlp.py > gpurun_out/r2h_diag_mlp.jsonl 2>&1; rc=$?
cat gpurun_out/r2h_diag_mlp.jsonl | cut -c1-220
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in bf16 fp32; do
  timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision $prec >> gpurun_out/r2h_kbench_mlp.jsonl || exit $?
done
cat gpurun_out/r2h_kbench_mlp.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2h_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2h_pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/r2h_counters.txt 2>&1 || echo "list rc=$?"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2h_prof_mlp -o mlp -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 10 --precision bf16 > gpurun_out/r2h_rocprof_mlp.log 2>&1 || echo "rocprof rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/r2h_pmc_tree -o tree --output-format csv -- python scripts/kbench.py --iters 3 > gpurun_out/r2h_pmc_tree.log 2>&1 || echo "pmc rc=$?"
find gpurun_out/r2h_prof_mlp gpurun_out/r2h_pmc_tree -name "*.csv" | head
