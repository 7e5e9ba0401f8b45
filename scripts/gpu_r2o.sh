#!/bin/bash
# round-2 GPU session O: reg MLP kernel after the loop vmcnt fix
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -q --timeout 120 --timeout-method thread > gpurun_out/r2o_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2o_pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 20 --precision bf16 --mlp-kernel reg >> gpurun_out/r2o_kbench.jsonl || exit $?
timeout -k 10 120 python -u scripts/kbench.py --model mlp --features 64 --rows 4194304 --iters 20 --precision bf16 --mlp-kernel reg >> gpurun_out/r2o_kbench.jsonl || exit $?
cut -c1-200 gpurun_out/r2o_kbench.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r2o_pmc_mlp -o mlp --output-format csv -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 3 --precision bf16 > gpurun_out/r2o_pmc_mlp.log 2>&1 || echo "pmc rc=$?"
echo done
