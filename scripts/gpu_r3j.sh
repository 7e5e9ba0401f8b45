set -o pipefail
mkdir -p gpurun_out/r3j
timeout -k 10 600 python -u -m pytest tests/test_math_context.py tests/test_wide_mlp.py tests/test_gpu_mlp.py tests/test_gpu_kernels.py tests/test_gpu_hybrid.py tests/test_gpu_segmented.py tests/test_design.py tests/test_gpu_surface.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3j/pytest.log 2>&1 || { tail -40 gpurun_out/r3j/pytest.log; exit 1; }
tail -1 gpurun_out/r3j/pytest.log
for M in gbdt rf; do
  for S in lockstep refill; do
    timeout -k 10 120 python -u scripts/kbench.py --model $M --trees 300 --depth 14 --p-split 0.85 --layout pointer --pointer-schedule $S --iters 10 >> gpurun_out/r3j/kbench.jsonl 2>> gpurun_out/r3j/kbench.err || exit 1
  done
done
for IMPL in wide gemm; do
  timeout -k 10 180 python -u scripts/kbench.py --model mlp --features 64 --hidden 1024,1024 --precision bf16 --mlp-impl $IMPL --rows 1048576 --iters 10 >> gpurun_out/r3j/kbench.jsonl 2>> gpurun_out/r3j/kbench.err || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3j/kbench.jsonl"):
    d = json.loads(l)
    print(d["model"], d.get("plan"), d["layout"], d.get("pointer_schedule"), round(d["ms"], 3), d.get("tflops"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j/prof_mlp -o mlp -- python3 scripts/kbench.py --model mlp --features 64 --hidden 1024,1024 --precision bf16 --mlp-impl wide --rows 1048576 --iters 5 > gpurun_out/r3j/prof_mlp.log 2>&1 || { tail -20 gpurun_out/r3j/prof_mlp.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace -d gpurun_out/r3j/pmc_mlp -o pmc -- python3 scripts/kbench.py --model mlp --features 64 --hidden 1024,1024 --precision bf16 --mlp-impl wide --rows 1048576 --iters 2 > gpurun_out/r3j/pmc_mlp.log 2>&1 || { tail -20 gpurun_out/r3j/pmc_mlp.log; exit 1; }
echo done
