#!/bin/bash
# round-2 GPU session AF: deep (unpadded) random forests on the pointer kernel — how far from
# the perfect-layout kernels are sklearn-style max_depth=None forests?
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_segmented.py tests/test_gpu_wide_modes.py tests/test_tree_shard_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r2af_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2af_pytest.log | tail -5; if [ $rc -gt 1 ]; then exit $rc; fi
mkdir -p gpurun_out
for a in "--depth 12 --trees 100" "--depth 16 --trees 100" "--depth 10 --trees 100 --layout pointer" "--depth 14 --trees 300"; do
  timeout -k 10 300 python -u scripts/kbench.py --model rf --rows 1048576 --iters 5 $a > gpurun_out/r2af_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2af_tmp.json')); print(repr(sys.argv[1]), round(d['ms'],3), 'ms', d['layout'], d['chunk_trees'], d['variant'])" "$a" | tee -a gpurun_out/r2af_kbench.txt
done
echo done
