set -o pipefail
# r5o: gemm8p (asm LDS-DMA staging) + persistent fused head: GPU tests, interleaved A/B, MLP kernel stats, PMC
O=gpurun_out/r5o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_wide_mlp.py -m gpu -k "persistent or wide_gemm_kernels or row_segment or phase_interleaved or fused_output" -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=1024,1024,1024,1024 FLAGS=0x1000,0,0x2000 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab -o k -- python3 scripts/gemm8p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep hidden $O/ab.log
python3 scripts/gemm8p_ab_parse.py $O/ab/k_kernel_trace.csv 3 > $O/ab_summary.json
HIDDEN=1024,1024,1024 FUSE_HEAD=1 FLAGS=0x1000,0 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/abh -o k -- python3 scripts/gemm8p_ab.py > $O/abh.log 2>&1 || { tail -20 $O/abh.log; exit 1; }
grep hidden $O/abh.log
python3 scripts/gemm8p_ab_parse.py $O/abh/k_kernel_trace.csv 1 > $O/abh_summary.json
FUSE_INPUT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 scripts/mlp_prof.py > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
grep hidden $O/k.log
FUSE_INPUT=0 timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc -o p -- python3 scripts/mlp_prof.py > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo done
