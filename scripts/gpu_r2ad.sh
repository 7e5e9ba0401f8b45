#!/bin/bash
# round-2 GPU session AD: VOTE8 forests with class codes in the last-level metas (no leaf array,
# no leaf read) — tree GPU tests + kernel-only forest timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wide_modes.py tests/test_gpu_segmented.py tests/test_gpu_target.py -q --timeout 120 --timeout-method thread > gpurun_out/r2ad_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r2ad_pytest.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "--model rf --depth 8 --trees 500" "--model rf --depth 8 --trees 500 --missing 0.02" "--model rf --depth 6 --trees 500" ""; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 --tree-prof $a > gpurun_out/r2ad_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2ad_tmp.json')); p=d['mlp_prof']; print(repr(sys.argv[1]), round(d['ms'],4), 'ms', d['chunk_trees'], d['variant'], [round(x) for x in p['mean']] if p else None)" "$a" | tee -a gpurun_out/r2ad_kbench.txt
done
timeout -k 10 300 python -u bench.py --model rf --steps 20 --warmup 3 > gpurun_out/r2ad_bench_rf.json 2> gpurun_out/r2ad_bench_rf.err || exit $?
cut -c1-300 gpurun_out/r2ad_bench_rf.json
echo done
