#!/bin/bash
# round-2 GPU session R: MFMA + LDS-B-operand micro-benchmark
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-value -Wno-unused-result scripts/ubench_mfma_lds.hip -o gpurun_out/ubench || exit 1
timeout -k 10 60 gpurun_out/ubench | tee gpurun_out/r2r_ubench.txt
