set -o pipefail
# Deep forests: fewer walks in flight per lane (2 / 4) for the pointer and SUPER layouts.
mkdir -p gpurun_out/r3aa
export HSA_ENABLE_IPC_MODE_LEGACY=0
for M in gbdt rf; do
  timeout -k 10 300 python -u scripts/deep_forest_sweep.py --model $M --configs pointer,pointer4,pointer2,super,super4,super2 > gpurun_out/r3aa/sweep_$M.jsonl 2> gpurun_out/r3aa/sweep_$M.err || { tail -20 gpurun_out/r3aa/sweep_$M.err; exit 1; }
done
python - <<'PY'
import json
for f in ("gbdt", "rf"):
    for l in open(f"gpurun_out/r3aa/sweep_{f}.jsonl"):
        d = json.loads(l)
        if "config" in d:
            print(f, d["config"], round(d["ms"], 3), d["valid_match"], "%.1e" % d["max_abs_err"])
PY
