#!/bin/bash
# round-2 GPU session U: rehearse the N>1 bench path with 2 ranks sharing the one GPU (gloo), then
# the 1-rank RCCL group (--force-dist), then the default 1-GPU bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
FJA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --rows 1048576 > gpurun_out/r2u_bench_gloo2.json 2> gpurun_out/r2u_bench_gloo2.err || { echo "gloo2 rc=$?"; tail -20 gpurun_out/r2u_bench_gloo2.err; exit 1; }
cut -c1-300 gpurun_out/r2u_bench_gloo2.json
timeout -k 10 300 python bench.py --force-dist --steps 10 --warmup 3 > gpurun_out/r2u_bench_rccl1.json 2> gpurun_out/r2u_bench_rccl1.err || { echo "rccl1 rc=$?"; tail -20 gpurun_out/r2u_bench_rccl1.err; exit 1; }
cut -c1-300 gpurun_out/r2u_bench_rccl1.json
timeout -k 10 300 python bench.py > gpurun_out/r2u_bench.json 2> gpurun_out/r2u_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r2u_bench.err; exit 1; }
cut -c1-300 gpurun_out/r2u_bench.json
