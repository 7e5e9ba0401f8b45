set -o pipefail
# r5av: randomized regression modelChain fuzz (ChainPlan) vs the oracle
O=gpurun_out/r5av
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_chain_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
