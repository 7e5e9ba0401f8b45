set -o pipefail
# r5r: gemm8p deferred half-tile epilogue (default) vs whole-tile (bit 15) vs gemm8_kernel: tests + interleaved A/B + kernel stats
O=gpurun_out/r5r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_wide_mlp.py -m gpu -k "persistent or row_segment or wide_gemm_kernels" -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=1024,1024,1024,1024 FLAGS=0x1000,0x8000,0 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab -o k -- python3 scripts/gemm8p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep hidden $O/ab.log
python3 scripts/gemm8p_ab_parse.py $O/ab/k_kernel_trace.csv 3 > $O/ab_summary.json
FUSE_INPUT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 scripts/mlp_prof.py > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
grep hidden $O/k.log
echo done
