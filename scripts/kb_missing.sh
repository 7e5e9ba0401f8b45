set -e
K="timeout -k 10 120 python scripts/kbench.py"
for m in 0 0.02 0.1; do $K --model gbdt --missing $m; done
$K --model gbdt --missing 0.02 --nan-mode off
