set -o pipefail
# r5z: early staging of the next tile's second slice (bit 17) on the asm-staged persistent kernel: tests + interleaved A/B
O=gpurun_out/r5z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_wide_mlp.py -m gpu -k "persistent_phase" -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIDDEN=1024,1024,1024,1024 FLAGS=0x1000,0,0x20000 ROUNDS=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab -o k -- python3 scripts/gemm8p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep hidden $O/ab.log
python3 scripts/gemm8p_ab_parse.py $O/ab/k_kernel_trace.csv 3 > $O/ab_summary.json && python3 -c "import json; d=json.load(open('$O/ab_summary.json')); [print(k, [(v[l]['median_us'], v[l]['min_us']) for l in sorted(v)]) for k,v in d.items()]"
echo done
