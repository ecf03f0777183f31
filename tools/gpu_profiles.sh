set -o pipefail
# round profiles: rocprofv3 trace/stats + PMC passes for C3 and C5 (tools/profile.sh), render SQ
# counters (tools/render_pmc.sh) and the per-FSM-phase profile (diagnostic build)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=${ROUND:-r03}
bash tools/profile.sh $R > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
WORKLOAD=c5 bash tools/profile.sh $R > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
bash tools/render_pmc.sh > gpurun_out/render_pmc.log 2>&1 || { tail -5 gpurun_out/render_pmc.log; exit 1; }
MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm.log 2>&1 || exit 1
echo profiles done
