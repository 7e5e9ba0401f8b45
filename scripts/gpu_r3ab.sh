set -o pipefail
# Text-source ingest with the memory-mapped parse; GPU surface + association/svm/hybrid spot tests.
mkdir -p gpurun_out/r3ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py --source text --rows 2097152 --steps 3 --warmup 1 --passes 2 --ingest-threads 16 > gpurun_out/r3ab/bench_text.json 2> gpurun_out/r3ab/bench_text.err || { tail -20 gpurun_out/r3ab/bench_text.err; exit 1; }
cut -c1-250 gpurun_out/r3ab/bench_text.json
timeout -k 10 300 python -u bench.py --source binary --steps 5 --warmup 2 --passes 4 > gpurun_out/r3ab/bench_binary.json 2> gpurun_out/r3ab/bench_binary.err || { tail -20 gpurun_out/r3ab/bench_binary.err; exit 1; }
cut -c1-250 gpurun_out/r3ab/bench_binary.json
