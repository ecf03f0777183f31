set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_quick.sh && bash tools/gpu_ds_profile.sh && LIBS="build/libmmx_lsoff.so" ROUNDS=3 STEPS=512 bash tools/ab.sh
