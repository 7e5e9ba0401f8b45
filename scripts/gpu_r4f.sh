set -o pipefail
# round 4: fused last-hidden + output layer (gemm8_kernel<true>) — wide MLP GPU tests, kernel
# stats of the 1024^3 MLP, plan vs hipBLASLt timing.
O=gpurun_out/r4f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_mlp.log 2>&1; rc=$?
tail -12 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python3 scripts/mlp_prof.py > $O/prof_mlp.log 2>&1; rc=$?
tail -2 $O/prof_mlp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/gemm_vs_blas.py > $O/gemm_vs_blas.jsonl 2> $O/gemm_vs_blas.err; rc=$?
cut -c1-200 $O/gemm_vs_blas.jsonl; exit $rc
