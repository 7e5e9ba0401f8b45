set -e
python scripts/kbench.py --model mlp --features 64
python scripts/kbench.py --model svm --features 16
python scripts/kbench.py --model rf --trees 500 --depth 8
python scripts/kbench.py --model kmeans
