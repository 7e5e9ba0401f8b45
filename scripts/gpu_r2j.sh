#!/bin/bash
# round-2 GPU session J: this box's H2D ceiling, wide-kernel ILP 8 vs 16, MLP PMC, bench variants,
# new/fixed GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/probe_h2d_sizes.py --rows 8388608 > gpurun_out/r2j_probe.jsonl || exit $?
cat gpurun_out/r2j_probe.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_target.py tests/test_gpu_svm_lr.py tests/test_gpu_segmented.py tests/test_gpu_mlp.py tests/test_gpu_wide_modes.py -v --timeout 120 --timeout-method thread > gpurun_out/r2j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/r2j_pytest.log | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
for a in "--ilp 8" "--ilp 16" "--ilp 16 --missing 0.02" "--ilp 16 --features 128" "--model rf --ilp 16"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a >> gpurun_out/r2j_kbench.jsonl || exit $?
done
cut -c1-160 gpurun_out/r2j_kbench.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH -d gpurun_out/r2j_pmc_mlp1 -o mlp --output-format csv -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 3 --precision bf16 > gpurun_out/r2j_pmc_mlp1.log 2>&1 || echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/r2j_pmc_mlp2 -o mlp --output-format csv -- python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 3 --precision bf16 > gpurun_out/r2j_pmc_mlp2.log 2>&1 || echo "pmc2 rc=$?"
for a in "" "--h2d-streams 2"; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 $a >> gpurun_out/r2j_bench.jsonl 2>> gpurun_out/r2j_bench.err || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/r2j_bench.jsonl"):
    d = json.loads(l)
    print(round(d["value"] / 1e6, 1), "M rec/s", d.get("h2d_gbps_effective"), d.get("kernel_ms_per_1M_rows"), d["config"].get("h2d_streams"))
PY
