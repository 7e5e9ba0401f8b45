set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3e/pytest_hybrid.log 2>&1 || { tail -30 gpurun_out/r3e/pytest_hybrid.log; exit 1; }
tail -2 gpurun_out/r3e/pytest_hybrid.log
for M in rf gbdt; do for H in 4 6 8; do timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout hybrid --head-depth $H --iters 10 >> gpurun_out/r3e/kbench.jsonl 2>> gpurun_out/r3e/kbench.err || exit 1; done; done
cut -c1-180 gpurun_out/r3e/kbench.jsonl
timeout -k 10 200 python -u bench.py --source binary --steps 5 --warmup 2 --passes 4 > gpurun_out/r3e/bench_binary.json 2> gpurun_out/r3e/bench_binary.err || { tail -20 gpurun_out/r3e/bench_binary.err; exit 1; }
cut -c1-400 gpurun_out/r3e/bench_binary.json
timeout -k 10 300 python -u bench.py --source text --rows 2097152 --steps 3 --warmup 1 --passes 2 --ingest-threads 16 > gpurun_out/r3e/bench_text.json 2> gpurun_out/r3e/bench_text.err || { tail -20 gpurun_out/r3e/bench_text.err; exit 1; }
cut -c1-400 gpurun_out/r3e/bench_text.json
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt > gpurun_out/r3e/per_record.jsonl 2> gpurun_out/r3e/per_record.err || { tail -20 gpurun_out/r3e/per_record.err; exit 1; }
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model kmeans >> gpurun_out/r3e/per_record.jsonl 2>> gpurun_out/r3e/per_record.err
timeout -k 10 200 python -u scripts/per_record_bench.py --device cuda --rows 2000000 --model gbdt --api to_batches >> gpurun_out/r3e/per_record.jsonl 2>> gpurun_out/r3e/per_record.err
cat gpurun_out/r3e/per_record.jsonl
