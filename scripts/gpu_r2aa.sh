#!/bin/bash
# round-2 GPU session AA: rocprofv3 evidence for the round's kernels — kernel-trace stats of the
# DSL bench (all kernels of an end-to-end run), PMC passes for the tree kernel (dynamic batches),
# the matrix-core SVM kernel and the bf16 MLP kernel
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r2aa_bench_stats -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 > gpurun_out/r2aa_bench.json 2> gpurun_out/r2aa_bench.err || { echo "bench stats rc=$?"; tail -5 gpurun_out/r2aa_bench.err; exit 1; }
cut -c1-300 gpurun_out/r2aa_bench.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r2aa_pmc_tree -o tree --output-format csv -- python scripts/kbench.py --iters 3 > gpurun_out/r2aa_pmc_tree.log 2>&1 || echo "pmc tree rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r2aa_pmc_svm -o svm --output-format csv -- python scripts/kbench.py --model svm --iters 3 > gpurun_out/r2aa_pmc_svm.log 2>&1 || echo "pmc svm rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r2aa_pmc_mlp -o mlp --output-format csv -- python scripts/kbench.py --model mlp --features 64 --precision bf16 --iters 3 > gpurun_out/r2aa_pmc_mlp.log 2>&1 || echo "pmc mlp rc=$?"
ls -R gpurun_out | grep -c csv
echo done
