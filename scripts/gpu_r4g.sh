set -o pipefail
# round 4: multi-segment pointer launch (segmented plans: 2 launches per batch), LDS-staged epilogue
# of small-K GEMM layers; GPU tests + kernel traces of the segmented batch and the 1024^3 MLP.
O=gpurun_out/r4g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_segmented.py tests/test_segmented.py tests/test_wide_mlp.py tests/test_gpu_mlp.py tests/test_gpu_hybrid.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_seg -o seg -- python3 scripts/seg_prof.py > $O/prof_seg.log 2>&1; rc=$?
grep '^\[' $O/prof_seg.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python3 scripts/mlp_prof.py > $O/prof_mlp.log 2>&1; rc=$?
grep '^{' $O/prof_mlp.log | tail -1; exit $rc
