#!/bin/bash
# round-2 GPU session AC: levels 0-1 of the dynamic-batch walks from global head loads (11 LDS
# reads per depth-6 fp32 walk instead of 13) — tree GPU tests + kernel-only timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py tests/test_gpu_segmented.py tests/test_gpu_target.py -q --timeout 120 --timeout-method thread > gpurun_out/r2ac_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2ac_pytest.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "" "--precision fp8" "--missing 0.02" "--depth 8 --trees 500" "--features 48"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 --tree-prof $a > gpurun_out/r2ac_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2ac_tmp.json')); p=d['mlp_prof']; print(repr(sys.argv[1]), round(d['ms'],4), 'ms', d['chunk_trees'], d['variant'], [round(x) for x in p['mean']] if p else None)" "$a" | tee -a gpurun_out/r2ac_kbench.txt
done
echo done
