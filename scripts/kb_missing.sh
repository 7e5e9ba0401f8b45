set -e
K="timeout -k 10 120 python scripts/kbench.py"
for c in 0 64 48 32; do
  $K --model gbdt --missing 0 --nan-mode off --max-chunk-trees $c
  $K --model gbdt --missing 0 --max-chunk-trees $c
  $K --model gbdt --missing 0.02 --max-chunk-trees $c
done
$K --model gbdt --missing 0.02 --nan-mode off
