#!/bin/bash
# r05: C5 (cameras) A/B of the step-kernel layout and the render z-buffer layout: product (128 rows,
# 10 envs/CU, render stride Sg + 4), l192r (192 rows, 8/CU, new render), l192 (192 rows, old render)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
WORKLOAD=c5 STEPS=128 LIBS="build/libmmx_l192r.so build/libmmx_l192.so" ROUNDS=3 bash tools/ab.sh
timeout -k 10 500 bash tools/render_pmc.sh > gpurun_out/render_pmc.log 2>&1 || { tail -5 gpurun_out/render_pmc.log; exit 1; }
python3 tools/render_pmc.py --round r05 && mkdir -p gpurun_out/box_profiles && cp profiles/r05_render_pmc.json profiles/pmc_render.json gpurun_out/box_profiles/
