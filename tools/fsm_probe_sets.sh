set -o pipefail
# per-FSM-state phase / sub-phase profile for each probe build build/libmmx_prof<P>.so (diagnostic)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for P in ${PROBE_SETS:-1 3 5 6 8 9 10}; do
  MMX_PROFILE=1 MMX_LIB_PATH=build/libmmx_prof$P.so timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_set$P.log 2>&1 || exit 1
  cp gpurun_out/probe_prof.json gpurun_out/fsm_set$P.json
done
echo done
