#!/bin/bash
# Diagnostic: per-phase and sub-phase shader-clock breakdown for probe sets (1 solver,
# 2 collision, 3 constraints, ...).  Uses prebuilt build/libmmx_prof<P>.so (built on the CPU
# host: MMX_PROBE=<P> _build.build(profile=True)); writes gpurun_out/probe_set<P>.json.
set -e
for P in ${PROBE_SETS:-1 2 3}; do
  MMX_PROFILE=1 MMX_LIB_PATH=build/libmmx_prof$P.so timeout -k 10 300 python tools/gpu_probe.py speed \
    > gpurun_out/probe_set$P.log 2>&1
  cp gpurun_out/probe_prof.json gpurun_out/probe_set$P.json
done
