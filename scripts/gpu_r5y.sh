set -o pipefail
# r5y: packed bf16 conversion in the epilogues: wide-MLP GPU tests + A/B + MLP kernel stats
O=gpurun_out/r5y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=1024,1024,1024,1024 FLAGS=0x1000,0,0x2000 ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab -o k -- python3 scripts/gemm8p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep hidden $O/ab.log
python3 scripts/gemm8p_ab_parse.py $O/ab/k_kernel_trace.csv 3 > $O/ab_summary.json && cat $O/ab_summary.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, [v[l]['median_us'] for l in sorted(v)]) for k,v in d.items()]"
FUSE_INPUT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 scripts/mlp_prof.py > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
grep hidden $O/k.log
echo done
