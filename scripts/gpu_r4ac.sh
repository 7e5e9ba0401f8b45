set -o pipefail
# end-of-round numbers at HEAD: --models 64, --source text, 100-class wide SVM, kernel stats of the headline bench
O=gpurun_out/r4ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py --models 64 --steps 10 --warmup 2 --passes 8 > $O/bench_models64.json 2> $O/bench_models64.err || { tail -20 $O/bench_models64.err; exit 1; }
tail -c 200 $O/bench_models64.json; echo
timeout -k 10 400 python -u bench.py --source text --steps 4 --warmup 1 --passes 2 --ingest-threads 16 > $O/bench_text.json 2> $O/bench_text.err || { tail -20 $O/bench_text.err; exit 1; }
tail -c 200 $O/bench_text.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 3 --warmup 1 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo done
