#!/bin/bash
# round-2 GPU session S: why fp8 leaves are slower than fp32 in the wide tree kernel
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for a in "--precision fp8" "--precision fp8 --max-chunk-trees 64" "--precision fp8 --max-chunk-trees 32" "--max-chunk-trees 32" "--precision fp8 --nan-mode off" "--nan-mode off"; do
  timeout -k 10 120 python -u scripts/kbench.py --rows 1048576 --iters 20 $a > gpurun_out/r2s_tmp.json || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r2s_tmp.json')); print(sys.argv[1], round(d['ms'],3), 'ms', d['chunk_trees'], d['variant'])" "$a" | tee -a gpurun_out/r2s_kbench.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r2s_pmc8 -o t --output-format csv -- python scripts/kbench.py --iters 3 --precision fp8 > gpurun_out/r2s_pmc8.log 2>&1 || echo "pmc rc=$?"
python - <<'PY'
import csv, collections
d = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r2s_pmc8/t_counter_collection.csv")):
    if "tree_perfect" in r["Kernel_Name"]:
        d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"]); d[r["Dispatch_Id"]]["k"] = r["Kernel_Name"][:90]
print(list(d.values())[-1])
PY
