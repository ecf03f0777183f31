#!/bin/bash
# r05: contact parameters computed once per contact and exchanged over ds_bpermute (product) vs per
# row (cps0): GPU suite, C3 A/B, 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_cps.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_cps.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_cps.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_cps0.so" ROUNDS=3 bash tools/ab.sh
