#!/bin/bash
# r05: longest-first order by FSM phase class (product) vs by the last substep's constraint rows
# (build/libmmx_clsrows.so), C3 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="build/libmmx_clsrows.so" ROUNDS=3 timeout -k 10 600 bash tools/ab.sh || exit 1
cp gpurun_out/ab/report.json gpurun_out/ab_clsrows_c3.json
LIBS="build/libmmx_clsrows.so" WORKLOAD=c5 STEPS=128 ROUNDS=3 timeout -k 10 600 bash tools/ab.sh || exit 1
cp gpurun_out/ab/report.json gpurun_out/ab_clsrows_c5.json
