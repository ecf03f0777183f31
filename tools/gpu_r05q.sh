#!/bin/bash
# r05: 11 envs per CU (9-float LDS contacts, the general Cholesky's transpose in HBM): full GPU suite
# with margins, then C3 A/B against the 10-per-CU build (p10 = HEAD), 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_11cu.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_11cu.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_11cu.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_p10.so" ROUNDS=3 bash tools/ab.sh
