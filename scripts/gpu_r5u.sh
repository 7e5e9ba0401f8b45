set -o pipefail
# r5u: gemm8p routed for every K >= 128 (and the fused head at any K): wide-MLP GPU tests, A/Bs, MLP kernel stats
O=gpurun_out/r5u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread -rf --durations=15 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -22 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=256,256,448,2048,1024 FLAGS=0x1000,0 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/mix -o k -- python3 scripts/gemm8p_ab.py > $O/mix.log 2>&1 || { tail -20 $O/mix.log; exit 1; }
grep hidden $O/mix.log
FUSE_INPUT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 scripts/mlp_prof.py > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
grep hidden $O/k.log
echo done
