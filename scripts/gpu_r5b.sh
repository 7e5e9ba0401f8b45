set -o pipefail
# r5b: device-counted grouped path (count + place + ONE grouped tree launch per config per slice)
O=gpurun_out/r5b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_mixed_models.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
FJA_PROFILE=2 timeout -k 10 400 python -u bench.py --models 64 --steps 8 --warmup 2 --passes 8 > $O/bench_models64.json 2> $O/bench_models64.err || { tail -20 $O/bench_models64.err; exit 1; }
tail -c 300 $O/bench_models64.json; echo
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_models64 -o m64 -- python3 bench.py --models 64 --steps 3 --warmup 1 --passes 4 > $O/prof_models64.log 2>&1 || { tail -20 $O/prof_models64.log; exit 1; }
echo done
