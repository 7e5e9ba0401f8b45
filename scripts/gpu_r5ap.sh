set -o pipefail
# r5ap: randomized RegressionModel design fuzz (categorical predictors, terms, exponents, links)
O=gpurun_out/r5ap
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_design_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
