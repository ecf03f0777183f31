#!/bin/bash
# Diagnostic: per-phase and sub-phase shader-clock breakdown for probe sets (1 solver,
# 5 narrowphase, 9 Cholesky, 10 line search, 12 row-count distribution, ...).  Uses prebuilt
# build/libmmx_prof<P>.so (built on the CPU host: python tools/build_probes.py <P>...); writes
# gpurun_out/probe_set<P>.json.
set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for P in ${PROBE_SETS:-1 2 3}; do
  WHAT=speed
  [ "$P" = "12" ] && WHAT=nefc
  MMX_PROFILE=1 MMX_LIB_PATH=build/libmmx_prof$P.so timeout -k 10 300 python tools/gpu_probe.py $WHAT \
    > gpurun_out/probe_set$P.log 2>&1
  cp gpurun_out/probe_prof.json gpurun_out/probe_set$P.json
done
