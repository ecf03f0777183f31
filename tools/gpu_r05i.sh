#!/bin/bash
# r05: C5 (cameras) A/B of the step-kernel layout and the render z-buffer layout: product (128 rows,
# 10 envs/CU, render stride Sg + 4), l192r (192 rows, 8/CU, new render), l192 (192 rows, old render)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
WORKLOAD=c5 STEPS=128 LIBS="build/libmmx_l192r.so build/libmmx_l192.so" ROUNDS=3 bash tools/ab.sh
