set -o pipefail
# r5l: persistent gemm8p with counted epilogue stores + asm-LDS epilogue: bit identity, kernel A/B (K=1024 and K=4096 layers), PMC
O=gpurun_out/r5l
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_wide_mlp.py -m gpu -k "persistent or wide_gemm_kernels or row_segment or phase_interleaved" -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 0x1000 0; do
  HIDDEN=1024,1024,4096,1024 ITERS=3 FUSE_INPUT=0 FUSE_HEAD=0 GEMM_FLAGS=$F timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/k_$F -o k -- python3 scripts/mlp_prof.py > $O/k_$F.log 2>&1 || { tail -20 $O/k_$F.log; exit 1; }
  grep hidden $O/k_$F.log || true
done
FUSE_INPUT=0 FUSE_HEAD=0 timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc -o p -- python3 scripts/mlp_prof.py > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo done
