set -e
python scripts/kbench.py --model pcie --iters 10
for m in 0 0.02; do
  python scripts/kbench.py --missing $m --variant wide
  python scripts/kbench.py --missing $m --variant narrow --lds-budget 49152
done
python scripts/kbench.py --model gbdt-binary
python scripts/kbench.py --depth 8 --trees 500
python scripts/kbench.py --model rf --trees 500 --depth 8
python scripts/kbench.py --features 64 --trees 1000
