set -e
K="timeout -k 10 120 python scripts/kbench.py"
$K --model gbdt --missing 0
$K --model gbdt --missing 0.02
$K --model gbdt --missing 0.02 --nan-mode off
$K --model gbdt --missing 0 --nan-mode off
$K --model gbdt --depth 8 --trees 500 --missing 0
$K --model gbdt --depth 8 --trees 500 --missing 0.02
$K --model gbdt-binary --missing 0
