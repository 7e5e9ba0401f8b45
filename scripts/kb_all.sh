# Kernel-only (HBM-resident records) numbers for every model family, one JSON line each.
set -e
K="timeout -k 10 120 python scripts/kbench.py"
$K --model gbdt
$K --model gbdt --missing 0.02
$K --model gbdt-binary
$K --model rf --trees 500 --depth 8
$K --model mlp --features 64
$K --model svm --features 16
$K --model lr
$K --model kmeans
$K --model kmeans-big --clusters 256 --features 64
