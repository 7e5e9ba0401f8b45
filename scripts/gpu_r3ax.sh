set -o pipefail
# the driver's launch shape on one card: torchrun with 1 rank (plain N = 1 path), then --force-dist (1-rank RCCL group through the N > 1 GatherSink path).
mkdir -p gpurun_out/r3ax
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/r3ax/bench_torchrun1.json 2> gpurun_out/r3ax/bench_torchrun1.err || { tail -20 gpurun_out/r3ax/bench_torchrun1.err; exit 1; }
cut -c1-300 gpurun_out/r3ax/bench_torchrun1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --steps 10 --warmup 2 --force-dist > gpurun_out/r3ax/bench_torchrun1_forcedist.json 2> gpurun_out/r3ax/bench_torchrun1_forcedist.err || { tail -20 gpurun_out/r3ax/bench_torchrun1_forcedist.err; exit 1; }
cut -c1-300 gpurun_out/r3ax/bench_torchrun1_forcedist.json
