#!/bin/bash
# r05: field-major LDS contact records (product) vs record-major (aos = HEAD): GPU suite + margins,
# C3 A/B with one PMC pass each (LDS bank conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_soa.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_soa.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_soa.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_aos.so" ROUNDS=3 PMC=1 bash tools/ab.sh
