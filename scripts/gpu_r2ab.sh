#!/bin/bash
# round-2 GPU session AB: vectorised, bank-conflict-free row staging (wide tree kernel + the
# shared stage_rows_T of the linear / cluster / SVM / derive / narrow tree kernels): full GPU
# suite, then kernel-only timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2ab_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2ab_pytest_gpu.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--precision fp8" "--features 128" "--missing 0.02" "--model rf --depth 8 --trees 500" "--model svm" "--model kmeans-big" "--model lr"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 --tree-prof $a > gpurun_out/r2ab_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2ab_tmp.json')); p=d['mlp_prof']; print(repr(sys.argv[1]), round(d['ms'],4), 'ms', d['chunk_trees'], d['variant'], [round(x) for x in p['mean']] if p else None)" "$a" | tee -a gpurun_out/r2ab_kbench.txt
done
echo done
