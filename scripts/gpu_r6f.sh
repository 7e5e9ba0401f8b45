set -o pipefail
# r6f: round-end smoke + bench N=1 + kernel stats of the bench + host rates (native walk).
O=gpurun_out/r6f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['n_gpus'], d['check'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cp "$(find $O/prof -name "*kernel_stats.csv" -print -quit)" $O/bench_kernel_stats.csv
head -8 $O/bench_kernel_stats.csv
timeout -k 10 300 python3 scripts/host_rate.py > $O/host_rate.json 2> $O/host_rate.err || { tail -20 $O/host_rate.err; exit 1; }
cat $O/host_rate.json
lscpu | grep -E "Model name|^CPU\(s\)|Flags" | cut -c1-200 > $O/cpu.txt
cat $O/cpu.txt
