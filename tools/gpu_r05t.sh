#!/bin/bash
# r05: 11 envs per CU for real (14,080 B: 8-float contacts with the geoms in the key word, warm start in
# E.x, cube mass entries as constants, 144-pair broadphase list; the LDS is allocated in 1,280-B blocks):
# GPU suite with margins, C3 A/B against HEAD (10 per CU), LDS residency probe
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib/lds_occ > gpurun_out/lds_occ.json 2> gpurun_out/lds_occ.err || exit 1
MMX_MARGINS_OUT=gpurun_out/parity_margins_11b.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_11b.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_11b.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_p10b.so" ROUNDS=3 bash tools/ab.sh
