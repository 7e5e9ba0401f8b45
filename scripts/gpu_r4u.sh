set -o pipefail
# wide SVM up to 256 classes: GPU tests, then wide kernel vs library GEMMs at 100 classes
O=gpurun_out/r4u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_svm_lr.py -x -q --timeout 180 --timeout-method thread -rf > $O/pytest_svm.log 2>&1 || { tail -30 $O/pytest_svm.log; exit 1; }
tail -3 $O/pytest_svm.log
for impl in wide gemm; do
  timeout -k 10 200 python -u scripts/kbench.py --model svm --classes 100 --n-sv 256 --features 32 --rows 262144 --iters 10 --svm-impl $impl > $O/kbench_svm100_$impl.json 2> $O/kbench_svm100_$impl.err || { tail -20 $O/kbench_svm100_$impl.err; exit 1; }
  tail -c 400 $O/kbench_svm100_$impl.json; echo
done
