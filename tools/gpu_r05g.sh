#!/bin/bash
# r05: render z-buffer stride Sg + 4 with b128 tile reads (product) against the r04 layout (rold):
# render tests, isolated render time + one SQ pass each (tools/render_sweep.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_render.py tests/test_png.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/gpu_tests_render.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_render.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_rold.so" bash tools/render_sweep.sh
