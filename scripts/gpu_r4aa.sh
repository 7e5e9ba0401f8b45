set -o pipefail
# transposed stores in the two-buffer bf16 kernel (K = 128 .. 448 layers): GPU bit-identity tests,
# then a 128-input 1024-1024 MLP kernel-only A/B (flag 0x100 = direct stores)
O=gpurun_out/r4aa
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_wide_mlp.py -m gpu -x -q --timeout 180 --timeout-method thread -rf -k "transposed" > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -2 $O/pytest_mlp.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in 0x100 0; do
  env FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=$f N_FEATURES=100 HIDDEN=1024,1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_$f -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_$f.log 2>&1 || exit 1
  grep '^{' $O/mlp_$f.log | tail -1
done
echo done
