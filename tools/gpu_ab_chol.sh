set -o pipefail
# contact A/B of the lane-quad box-box (prequad vs working tree), then the FSM-profile / bench A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BASE=build/libmmx_prequad.so bash tools/gpu_contact_ab.sh > gpurun_out/cab.txt 2>&1 || exit 1
bash tools/gpu_ab_fsm.sh
