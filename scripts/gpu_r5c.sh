set -o pipefail
# r5c: LDS-resident deep-forest walk (tree_lds.hip) — parity, then 300 x depth-14 kernel sweep; host NUMA probe
O=gpurun_out/r5c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_lds_forest.py -m gpu -x -v --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u scripts/deep_forest_sweep.py --model gbdt --configs pointer,lds > $O/sweep_gbdt.jsonl 2> $O/sweep_gbdt.err || { tail -20 $O/sweep_gbdt.err; exit 1; }
cat $O/sweep_gbdt.jsonl
timeout -k 10 400 python -u scripts/deep_forest_sweep.py --model rf --configs pointer,lds > $O/sweep_rf.jsonl 2> $O/sweep_rf.err || { tail -20 $O/sweep_rf.err; exit 1; }
cat $O/sweep_rf.jsonl
timeout -k 10 200 python -u scripts/numa_read_probe.py > $O/numa_probe.json 2> $O/numa_probe.err || { tail -20 $O/numa_probe.err; exit 1; }
cat $O/numa_probe.json
