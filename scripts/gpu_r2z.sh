#!/bin/bash
# round-2 GPU session Z: dynamic tree batches (slot order independent of chunk size) + MFMA SVM
# kernel — tree/SVM GPU tests, kernel-only timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py tests/test_gpu_segmented.py tests/test_gpu_svm_lr.py -q --timeout 120 --timeout-method thread > gpurun_out/r2z_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2z_pytest.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--precision fp8" "--missing 0.02" "--model rf --depth 8 --trees 500" "--features 128" "--model svm"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 --tree-prof $a > gpurun_out/r2z_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2z_tmp.json')); p=d['mlp_prof']; print(repr(sys.argv[1]), round(d['ms'],3), 'ms', d['chunk_trees'], d['variant'], [round(x) for x in p['mean']] if p else None)" "$a" | tee -a gpurun_out/r2z_kbench.txt
done
echo done
