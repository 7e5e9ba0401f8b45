set -o pipefail
# round 4: wave-private LDS epilogue (16-byte stores) of the bf16 hidden layers, RANK3 with LDS-staged
# rank search + 2-round rank reads: GPU tests, MLP kernel stats per variant, deep-forest sweep.
O=gpurun_out/r4k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_rank3.py tests/test_wide_mlp.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; ok $rc || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model gbdt --configs pointer,rank3,rank3_4 > $O/sweep_gbdt.jsonl 2> $O/sweep_gbdt.err; rc=$?
cut -c1-160 $O/sweep_gbdt.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model rf --configs pointer,rank3 > $O/sweep_rf.jsonl 2> $O/sweep_rf.err; rc=$?
cut -c1-160 $O/sweep_rf.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_$n -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_$n.log 2>&1 || return 1
  grep '^{' $O/mlp_$n.log | tail -1
}
run direct FUSE_INPUT=0 FUSE_HEAD=1 GEMM_FLAGS=0x20 && run wave FUSE_INPUT=0 FUSE_HEAD=1 && run base FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=0x60 || exit 1
echo done
