#!/bin/bash
# round-2 GPU session X: tree traversal variants (plain / register heads / pipelined half-batches)
# A/B on the depth-6 1000-tree GBDT + per-wave phase timers; tree GPU tests first
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py -q --timeout 120 --timeout-method thread > gpurun_out/r2x_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2x_pytest.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for rh in off auto; do for tp in 0 1 2; do for extra in "" "--precision fp8" "--model rf --depth 8 --trees 500"; do
  a="--reg-head $rh --tree-pipe $tp $extra"
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 --tree-prof $a > gpurun_out/r2x_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2x_tmp.json')); p=d['mlp_prof']; print(repr(sys.argv[1]), round(d['ms'],3), 'ms', d['variant'], [round(x) for x in p['mean']] if p else None)" "$a" | tee -a gpurun_out/r2x_kbench.txt
done; done; done
echo done
