set -o pipefail
# Host overhead of the small-batch predict path (cProfile); text-source ingest after the read-window
# rewrite.
mkdir -p gpurun_out/r3y
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/profile_predict.py > gpurun_out/r3y/profile_predict.txt 2> gpurun_out/r3y/profile_predict.err || { tail -30 gpurun_out/r3y/profile_predict.err; exit 1; }
head -45 gpurun_out/r3y/profile_predict.txt
timeout -k 10 400 python -u bench.py --source text --rows 2097152 --steps 3 --warmup 1 --passes 2 --ingest-threads 16 > gpurun_out/r3y/bench_text.json 2> gpurun_out/r3y/bench_text.err || { tail -20 gpurun_out/r3y/bench_text.err; exit 1; }
cut -c1-250 gpurun_out/r3y/bench_text.json
timeout -k 10 200 python -u scripts/probe_splits.py > gpurun_out/r3y/splits.jsonl 2> gpurun_out/r3y/splits.err || { tail -20 gpurun_out/r3y/splits.err; exit 1; }
cat gpurun_out/r3y/splits.jsonl
