set -o pipefail
# wide-layer GEMM: LDS swizzle variant A/B (one process, interleaved) + LDS / MFMA PMC of both variants.
mkdir -p gpurun_out/r3ak
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u scripts/gemm_ab.py > gpurun_out/r3ak/ab_bf16.jsonl 2> gpurun_out/r3ak/ab.err || { tail -20 gpurun_out/r3ak/ab.err; exit 1; }
PRECISION=fp32 VARIANTS=1,0x11 timeout -k 10 300 python -u scripts/gemm_ab.py > gpurun_out/r3ak/ab_fp32.jsonl 2>> gpurun_out/r3ak/ab.err || { tail -20 gpurun_out/r3ak/ab.err; exit 1; }
cat gpurun_out/r3ak/ab_bf16.jsonl gpurun_out/r3ak/ab_fp32.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for var in 0 0x10; do
  FJA_GEMM_FLAGS=$var ROUNDS=1 VARIANTS=$var timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r3ak/pmc_$var -o p --output-format csv -- python3 scripts/gemm_ab.py > gpurun_out/r3ak/pmc_$var.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/r3ak/pmc_$var.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r3ak/pmc_*/p_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "gemm_kernel<256" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, {k: f"{v:.3e}" for k, v in sorted(agg.items())})
PY
