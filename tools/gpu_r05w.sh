#!/bin/bash
# r05: the arm-coupled Cholesky's coupled-cube update reads the arm's 9 final values first (product)
# vs HEAD: GPU suite + margins, C3 A/B (3 rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_za.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_za.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_za.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_base.so" ROUNDS=3 bash tools/ab.sh
