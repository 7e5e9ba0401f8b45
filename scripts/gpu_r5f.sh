set -o pipefail
# r5f: K = 64 layer row-segment stores (gemm flag bit 10): bit identity + kernel stats A/B + PMC
O=gpurun_out/r5f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_wide_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread -rf -k "segment or transposed" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 0 0x400; do
  GEMM_FLAGS=$F timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$F -o k -- python3 scripts/mlp_prof.py > $O/k_$F.log 2>&1 || { tail -20 $O/k_$F.log; exit 1; }
  grep hidden $O/k_$F.log || true
  grep -h "k64p\|gemm8" $O/k_$F/k_kernel_stats.csv | cut -d, -f1-4
done
GEMM_FLAGS=0x400 timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_seg -o p -- python3 scripts/mlp_prof.py > $O/pmc_seg.log 2>&1 || { tail -20 $O/pmc_seg.log; exit 1; }
echo done
