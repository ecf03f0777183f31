#!/bin/bash
# r05: 96 LDS rows (12 envs per CU: 12,800 B; EPA polytope over the candidate list + 256 scratch
# floats) vs the 128-row product (which carries the EPA relocation too): GPU suite with both, C3 and
# C5 interleaved A/Bs
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="build/libmmx_l96.so" TESTS=1 ROUNDS=3 timeout -k 10 1000 bash tools/ab.sh || exit 1
cp gpurun_out/ab/report.json gpurun_out/ab_c3_report.json
LIBS="build/libmmx_l96.so" WORKLOAD=c5 STEPS=128 ROUNDS=2 timeout -k 10 600 bash tools/ab.sh || exit 1
cp gpurun_out/ab/report.json gpurun_out/ab_c5_report.json
