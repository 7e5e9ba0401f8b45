set -o pipefail
# r5q: final wide-MLP state (gemm8p + persistent fused head + nt K=64 stores): all wide/mlp GPU tests, kernel stats, PMC
O=gpurun_out/r5q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FUSE_INPUT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 scripts/mlp_prof.py > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
grep hidden $O/k.log
FUSE_INPUT=0 timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc -o p -- python3 scripts/mlp_prof.py > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo done
