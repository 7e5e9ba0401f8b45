set -o pipefail
mkdir -p gpurun_out/r3m
timeout -k 10 300 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3m/pytest.log 2>&1 || { tail -40 gpurun_out/r3m/pytest.log; exit 1; }
tail -1 gpurun_out/r3m/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m/prof_mlp -o mlp -- python3 scripts/kbench.py --model mlp --features 64 --hidden 1024,1024 --precision bf16 --mlp-impl wide --rows 1048576 --iters 5 > gpurun_out/r3m/prof_mlp.log 2>&1 || { tail -20 gpurun_out/r3m/prof_mlp.log; exit 1; }
grep '"model"' gpurun_out/r3m/prof_mlp.log || true
find gpurun_out/r3m/prof_mlp -name "*kernel_stats.csv" -exec cat {} \;
