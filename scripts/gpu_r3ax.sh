set -o pipefail
# the driver's N > 1 launch shape on one card: torchrun, 1 rank, RCCL group, library GatherSink.
mkdir -p gpurun_out/r3ax
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/r3ax/bench_torchrun1.json 2> gpurun_out/r3ax/bench_torchrun1.err || { tail -20 gpurun_out/r3ax/bench_torchrun1.err; exit 1; }
cut -c1-300 gpurun_out/r3ax/bench_torchrun1.json
