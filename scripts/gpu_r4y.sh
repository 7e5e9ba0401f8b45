set -o pipefail
# 1024^3 bf16 MLP after the transposed stores / persistent K = 64 layer / LDS input tables: kernel
# stats (final config) and MFMA-busy PMC (own pass, kernel trace only)
O=gpurun_out/r4y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
env FUSE_INPUT=0 FUSE_HEAD=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp_stats -o mlp -- python3 scripts/mlp_prof.py > $O/mlp_stats.log 2>&1 || { tail -20 $O/mlp_stats.log; exit 1; }
grep '^{' $O/mlp_stats.log | tail -1
env FUSE_INPUT=0 FUSE_HEAD=1 ITERS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/mlp_pmc -o pmc -- python3 scripts/mlp_prof.py > $O/mlp_pmc.log 2>&1 || { tail -20 $O/mlp_pmc.log; exit 1; }
grep '^{' $O/mlp_pmc.log | tail -1
for i in 1 2 3; do env FUSE_INPUT=0 FUSE_HEAD=1 ITERS=30 timeout -k 10 120 python3 scripts/mlp_prof.py 2>&1 | tail -1; done > $O/plain.jsonl || exit 1
cat $O/plain.jsonl
echo done
