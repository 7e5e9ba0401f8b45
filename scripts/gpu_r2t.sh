#!/bin/bash
# round-2 GPU session T: tree traversal with explicit per-level phases (fp8 + fp32)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py tests/test_gpu_segmented.py -q --timeout 120 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2t_pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--precision fp8" "--missing 0.02" "--model rf --depth 8 --trees 500" "--features 128" "--model gbdt-binary --precision fp8"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a > gpurun_out/r2t_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2t_tmp.json')); print(sys.argv[1], round(d['ms'],3), 'ms', d['chunk_trees'], d['variant'])" "$a" | tee -a gpurun_out/r2t_kbench.txt
done
