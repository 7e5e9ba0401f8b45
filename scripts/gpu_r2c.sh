#!/bin/bash
# round-2 GPU session C: H2D bandwidth vs buffer size / NUMA placement + bench step-size variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r2c_probe.jsonl; : > $out
for rows in 1048576 8388608; do
  for numa in auto none 0 1; do
    timeout -k 10 120 python -u scripts/probe_h2d_sizes.py --rows $rows --numa $numa >> $out 2>> gpurun_out/r2c_probe.err || echo "probe $rows $numa rc=$?"
  done
done
cat $out
for mode in "--rows 1048576 --api engine" "--rows 1048576" "--rows 8388608 --no-numa" "--rows 4194304" "--rows 8388608 --micro-batch 1048576"; do
  tag=$(echo "$mode" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 python -u bench.py $mode --check-rows 0 > gpurun_out/r2c_bench${tag}.json 2> gpurun_out/r2c_bench${tag}.err || { echo "bench $mode failed rc=$?"; tail -5 gpurun_out/r2c_bench${tag}.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,1), 'M rec/s', round(d['h2d_gbps_effective'],1), 'GB/s', d['config']['numa_node'])" gpurun_out/r2c_bench${tag}.json "$mode"
done
