set -e
python bench.py --steps 30 --check-rows 0 --latency-iters 5 > gpurun_out/b1.log 2>&1
python bench.py --steps 30 --check-rows 0 --latency-iters 5 --no-numa > gpurun_out/b2.log 2>&1
python bench.py --steps 30 --check-rows 0 --latency-iters 5 --micro-batch 131072 > gpurun_out/b3.log 2>&1
python bench.py --steps 30 --check-rows 0 --latency-iters 5 --micro-batch 524288 --pipeline-depth 3 > gpurun_out/b4.log 2>&1
python scripts/probe_pipe.py > gpurun_out/probe3.log 2>&1
for f in gpurun_out/b*.log; do echo $f; grep -o '"value": [0-9.]*\|ms_per_step": [0-9.]*\|numa_node": [0-9a-z]*\|host_submit_ms_per_step": [0-9.]*' $f; done
