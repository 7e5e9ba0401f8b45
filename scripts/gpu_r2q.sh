#!/bin/bash
# round-2 GPU session Q: reg MLP kernel counters (LDS pressure vs MFMA)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K="python scripts/kbench.py --model mlp --features 64 --rows 1048576 --iters 3 --precision bf16"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r2q_pmc1 -o p --output-format csv -- $K > gpurun_out/r2q_pmc1.log 2>&1 || echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_LDS SQ_WAVES -d gpurun_out/r2q_pmc2 -o p --output-format csv -- $K > gpurun_out/r2q_pmc2.log 2>&1 || echo "pmc2 rc=$?"
python - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/r2q_pmc*/p_counter_collection.csv")):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "mlp_reg" in r["Kernel_Name"]:
            d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    print(f, list(d.values())[-1] if d else None)
PY
