#!/bin/bash
# r05: per-FSM-phase profile of the 10-envs-per-CU layout (default probe build + sub-phase probe sets
# 1 solver, 5 collision, 9 Cholesky, 10 line search)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_default.log 2>&1 || { tail -5 gpurun_out/fsm_default.log; exit 1; }
cp gpurun_out/probe_prof.json gpurun_out/fsm_default.json
PROBE_SETS="1 5 9 10" bash tools/fsm_probe_sets.sh
