set -e
for v in valu mfma; do
  for kf in "64 32" "256 32" "256 64" "1024 64"; do
    set -- $kf
    timeout -k 10 120 python scripts/kbench.py --model kmeans-big --variant $v --clusters $1 --features $2 --iters 10
  done
done
