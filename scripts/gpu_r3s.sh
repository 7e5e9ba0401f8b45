set -o pipefail
# N>1 code path rehearsed on one GPU: 4 gloo ranks share the card (4 pinned shards, 4 concurrent
# H2D calibrations, per-rank NUMA binding, the library GatherSink over gloo); the 1-rank RCCL
# group; text-source ingest end to end.
mkdir -p gpurun_out/r3s
export HSA_ENABLE_IPC_MODE_LEGACY=0
FJA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 4 --warmup 2 --rows 1048576 --passes 4 > gpurun_out/r3s/bench_gloo4.json 2> gpurun_out/r3s/bench_gloo4.err || { echo "gloo4 rc=$?"; tail -30 gpurun_out/r3s/bench_gloo4.err; exit 1; }
cut -c1-400 gpurun_out/r3s/bench_gloo4.json
timeout -k 10 300 python bench.py --force-dist --steps 10 --warmup 3 > gpurun_out/r3s/bench_rccl1.json 2> gpurun_out/r3s/bench_rccl1.err || { echo "rccl1 rc=$?"; tail -20 gpurun_out/r3s/bench_rccl1.err; exit 1; }
cut -c1-300 gpurun_out/r3s/bench_rccl1.json
timeout -k 10 400 python -u bench.py --source text --rows 2097152 --steps 3 --warmup 1 --passes 2 --ingest-threads 16 > gpurun_out/r3s/bench_text.json 2> gpurun_out/r3s/bench_text.err || { tail -20 gpurun_out/r3s/bench_text.err; exit 1; }
cut -c1-300 gpurun_out/r3s/bench_text.json
