set -o pipefail
# r5aw: chain fuzz seeds whose segments have no inputs (the r5av fault: a 0-wide matrix handed to
# the tree kernel, now padded to one column)
O=gpurun_out/r5aw
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest "tests/test_chain_fuzz.py::test_random_chains_on_gpu[6]" "tests/test_chain_fuzz.py::test_random_chains_on_gpu[7]" "tests/test_chain_fuzz.py::test_random_chains_on_gpu[9]" -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
