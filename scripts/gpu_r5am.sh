set -o pipefail
# r5am: PMML 4.4 functions in the derive kernel (erf, standard normal CDF/PDF/IDF, hypot, atan2) + weightedSum ensembles
O=gpurun_out/r5am
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_derive.py tests/test_weighted_sum.py tests/test_design.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
