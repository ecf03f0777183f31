#!/bin/bash
# Diagnostic: per-phase and sub-phase shader-clock breakdown for probe sets 1..3
# (solver, collision, constraints).  Rebuilds libmmx_prof.so per set; writes gpurun_out/probe_set{N}.json.
set -e
for P in ${PROBE_SETS:-1 2 3}; do
  MMX_PROBE=$P python -c "from mujoco_manip_amd import _build; _build.build(force=True, profile=True)"
  MMX_PROFILE=1 timeout -k 10 300 python tools/gpu_probe.py speed > gpurun_out/probe_set$P.log 2>&1
  cp gpurun_out/probe_prof.json gpurun_out/probe_set$P.json
done
