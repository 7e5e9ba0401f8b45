#!/bin/bash
# round-2 GPU session B: DSL bench + engine bench + model modes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in "" "--api engine" "--model chain --precision fp8" "--model rf" "--model mlp"; do
  tag=$(echo "$mode" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 python -u bench.py $mode > gpurun_out/r2b_bench${tag}.json 2> gpurun_out/r2b_bench${tag}.err || { echo "bench $mode failed rc=$?"; tail -5 gpurun_out/r2b_bench${tag}.err; exit 1; }
  cat gpurun_out/r2b_bench${tag}.json
done
