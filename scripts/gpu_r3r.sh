set -o pipefail
# Wide SVM kernel (two chained f32 MFMA products): GPU tests, kernel-only vs the library-GEMM
# plan, MFMA-busy counters.
mkdir -p gpurun_out/r3r
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_svm_lr.py tests/test_gpu_kernels.py -k "svm or SVM" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3r/pytest.log 2>&1 || { tail -40 gpurun_out/r3r/pytest.log; exit 1; }
tail -1 gpurun_out/r3r/pytest.log
for IMPL in wide gemm; do
  for CFG in "--classes 12 --n-sv 1024 --features 64" "--classes 5 --n-sv 512 --features 32" "--classes 2 --n-sv 2048 --features 100"; do
    timeout -k 10 120 python -u scripts/kbench.py --model svm $CFG --svm-impl $IMPL --iters 10 >> gpurun_out/r3r/kbench.jsonl 2>> gpurun_out/r3r/kbench.err || { tail -20 gpurun_out/r3r/kbench.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3r/kbench.jsonl"):
    d = json.loads(l)
    print(d["plan"], d["features"], round(d["ms"], 3), d.get("tflops"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3r/pmc -o pmc -- python3 scripts/kbench.py --model svm --classes 12 --n-sv 1024 --features 64 --svm-impl wide --iters 3 > gpurun_out/r3r/pmc.log 2>&1 || { tail -20 gpurun_out/r3r/pmc.log; exit 1; }
ls gpurun_out/r3r/pmc
