#!/bin/bash
# round-2 GPU session W: register-head tree traversal (VAR_REG_HEAD) — tree GPU tests, then A/B
# kernel-only timings (auto vs --reg-head off) and a PMC pass
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py tests/test_gpu_segmented.py tests/test_gpu_target.py -q --timeout 120 --timeout-method thread > gpurun_out/r2w_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2w_pytest.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--reg-head off" "--precision fp8" "--precision fp8 --reg-head off" "--missing 0.02" "--model rf --depth 8 --trees 500" "--model rf --depth 8 --trees 500 --reg-head off" "--model gbdt-binary --precision fp8"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a > gpurun_out/r2w_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2w_tmp.json')); print(repr(sys.argv[1]), round(d['ms'],3), 'ms', d['chunk_trees'], d['variant'])" "$a" | tee -a gpurun_out/r2w_kbench.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/r2w_pmc_tree -o tree --output-format csv -- python scripts/kbench.py --iters 3 > gpurun_out/r2w_pmc_tree.log 2>&1 || echo "pmc tree rc=$?"
echo done
