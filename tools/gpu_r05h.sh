#!/bin/bash
# r05 evidence call: render z-buffer layout A/B (tools/gpu_r05g.sh), then the round's profiles
# (rocprof stats + PMC + extended SQ of C3, tools/profile.sh) and bench lines (tools/gpu_evidence.sh)
# of the 10-envs-per-CU product; box-side profiles/ outputs copied under gpurun_out/box_profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/box_profiles
bash tools/gpu_r05g.sh || exit 1
timeout -k 10 900 bash tools/profile.sh r05 > gpurun_out/profile_r05.log 2>&1 || { tail -20 gpurun_out/profile_r05.log; exit 1; }
cp profiles/r05_c3_* profiles/pmc_c3.json gpurun_out/box_profiles/ || exit 1
ROUND=r05 bash tools/gpu_evidence.sh || exit 1
