#!/bin/bash
# r05 end, part 1: GPU suite (with the parity margins), smoke(), C3 rocprof stats + PMC + extended SQ
# (tools/profile.sh), bench lines C3 (CPU baseline) / driver config / C2 / C5 (tools/gpu_evidence.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/box_profiles
MMX_MARGINS_OUT=gpurun_out/parity_margins_end.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_end.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_end.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1 || { tail -5 gpurun_out/smoke_end.log; exit 1; }
tail -1 gpurun_out/smoke_end.log
timeout -k 10 900 bash tools/profile.sh r05 > gpurun_out/profile_r05.log 2>&1 || { tail -20 gpurun_out/profile_r05.log; exit 1; }
cp profiles/r05_c3_* profiles/pmc_c3.json gpurun_out/box_profiles/ || exit 1
ROUND=r05 bash tools/gpu_evidence.sh
