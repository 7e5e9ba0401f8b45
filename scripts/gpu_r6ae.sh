set -o pipefail
# r6ae: the RCCL code path at N = 1 (1-rank RCCL group: replicated model load, all-gather sink).
O=gpurun_out/r6ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 bench.py --gpus 1 --steps 5 --warmup 2 --force-dist > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { tail -30 $O/bench_rccl1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_rccl1.json').read().strip().splitlines()[-1]); c=d['config']; print(d['value'], d['n_gpus'], c.get('parallelism'), c.get('allgather_sink'), d['check'])"
