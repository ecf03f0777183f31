set -o pipefail
# box-box lane-quad A/B: GPU suite on the working tree, bit-identity digests of base vs new,
# FSM phase profiles and interleaved bench (tools/gpu_ab_fsm.sh does the last two)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BASE=${BASE:-build/libmmx_base.so}
MMX_LIB_PATH=$BASE timeout -k 10 200 python -u tools/gpu_probe.py digest > gpurun_out/dig_base.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gpu_probe.py digest > gpurun_out/dig_new.log 2>&1 || exit 1
tail -3 gpurun_out/dig_base.log gpurun_out/dig_new.log
bash tools/gpu_ab_fsm.sh
