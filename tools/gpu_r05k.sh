#!/bin/bash
# r05: C5 A/B of layouts + render PMC (tools/gpu_r05i.sh), then the FSM phase profile of the
# 10-envs-per-CU layout (tools/gpu_r05j.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_r05i.sh || exit 1
bash tools/gpu_r05j.sh || exit 1
