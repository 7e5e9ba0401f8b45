set -o pipefail
# round 4: RANK3 deep-forest walk (3 levels per 16-byte record on threshold ranks) — GPU tests +
# the 300 x depth-14 sweep vs the pointer walk; 3-WG/CU first-layer GEMM — tests + MLP stats.
O=gpurun_out/r4h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_rank3.py tests/test_wide_mlp.py tests/test_gpu_segmented.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log; ok $rc || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model gbdt --configs pointer,rank3,rank3_4,rank3_16,auto > $O/sweep_gbdt.jsonl 2> $O/sweep_gbdt.err; rc=$?
cut -c1-220 $O/sweep_gbdt.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/deep_forest_sweep.py --model rf --configs pointer,rank3,auto > $O/sweep_rf.jsonl 2> $O/sweep_rf.err; rc=$?
cut -c1-220 $O/sweep_rf.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python3 scripts/mlp_prof.py > $O/prof_mlp.log 2>&1; rc=$?
grep "^{" $O/prof_mlp.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_mlp -o pmc -- python3 scripts/mlp_prof.py > $O/pmc_mlp.log 2>&1; rc=$?
grep '^{' $O/pmc_mlp.log | tail -1; exit $rc
