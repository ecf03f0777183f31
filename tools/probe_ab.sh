cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for L in $LIBS; do n=$(basename $L .so)
MMX_PROFILE=1 MMX_LIB_PATH=$L timeout -k 10 300 python tools/gpu_probe.py speed > gpurun_out/probe_$n.log 2>&1 || exit 1
cp gpurun_out/probe_prof.json gpurun_out/probe_$n.json; done
