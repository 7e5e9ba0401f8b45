#!/usr/bin/env bash
# One GPU session on the gpurun box: tests -> bench -> rocprof. Each GPU step has its own time
# limit; a fault/abort/timeout (rc >= 124 or signal) stops the session, ordinary test failures
# (rc 1) do not.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="${STEPS:-tests bench prof}"

fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log" | tee -a "$OUT/session.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}

if python -c "from flink_jpmml_amd.ops import _lib; import sys; sys.exit(0 if _lib.is_stale() else 1)"; then
  run build 600 python -c "import __graft_entry__ as g; g.build()"
fi
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps "${BENCH_STEPS:-20}" --warmup 3 ;;
    prof)
      mkdir -p "$OUT/prof"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" \
          -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --latency-iters 5 \
          > "$OUT/prof.log" 2>&1 ); rc=$?
      echo "=== prof rc=$rc" | tee -a "$OUT/session.log"
      if fatal $rc; then exit $rc; fi ;;
    kbench)
      run kbench 600 bash -c "${KBENCH_CMD:-python scripts/kbench.py}" ;;
    pmc)
      mkdir -p "$OUT/pmc"
      rocprofv3 -L > "$OUT/pmc/counters.txt" 2>&1 || true
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --pmc ${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY} \
          -d "$OUT/pmc" -o pmc --output-format csv -- python3 "$ROOT/scripts/kbench.py" --iters 3 ${KB_ARGS:-} \
          > "$OUT/pmc.log" 2>&1 ); rc=$?
      echo "=== pmc rc=$rc" | tee -a "$OUT/session.log"
      if fatal $rc; then exit $rc; fi ;;
    trace)
      mkdir -p "$OUT/trace"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
          -d "$OUT/trace" -o trace --output-format csv -- python3 "$ROOT/bench.py" --steps 4 --warmup 1 \
          --latency-iters 3 --check-rows 0 > "$OUT/trace.log" 2>&1 ); rc=$?
      echo "=== trace rc=$rc" | tee -a "$OUT/session.log"
      if fatal $rc; then exit $rc; fi ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "=== session done" | tee -a "$OUT/session.log"
