set -o pipefail
# per-kernel device time of the wide MLP (2048-2048 and 1024-1024-512), 2-buffer vs phase-interleaved hidden GEMM
mkdir -p gpurun_out/r3ao
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for hid in 2048,2048 1024,1024,512; do
  for var in 0 0x80; do
    tag=${hid//,/x}_$var
    HIDDEN=$hid ROUNDS=2 VARIANTS=$var timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ao/$tag -o k --output-format csv -- python3 scripts/gemm_ab.py > gpurun_out/r3ao/$tag.log 2>&1 || { echo "rc=$? $tag"; tail -5 gpurun_out/r3ao/$tag.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/r3ao/*/k_kernel_stats.csv")):
    print(f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "gemm" in n or "nn_prep" in n:
            print("   %-70s calls %5s avg_us %10.1f" % (n[:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
