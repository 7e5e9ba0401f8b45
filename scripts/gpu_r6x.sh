set -o pipefail
# r6x: deep forests END TO END through the DSL (pinned host records -> H2D -> LTOP walk -> host
# sink): 300 trees x depth 14, GBDT and RF, 1 GPU.
O=gpurun_out/r6x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gbdt rf; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 --model $m --trees 300 --depth 14 > $O/bench_$m.json 2> $O/bench_$m.err || { tail -30 $O/bench_$m.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['config'].get('rows_per_pass'), d['check'], d['config'].get('h2d_gbps_effective'))"
done
