set -o pipefail
# sanity of the final in-tree build: wide-MLP GPU tests + smoke()
O=gpurun_out/r4ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_wide_mlp.py tests/test_gpu_svm_lr.py -m gpu -x -q --timeout 180 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
