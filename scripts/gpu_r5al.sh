set -o pipefail
# r5al: discretized NaiveBayes inputs (BayesInput DerivedField) + scorecards through the device plans
O=gpurun_out/r5al
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_design.py tests/test_scorecard.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
