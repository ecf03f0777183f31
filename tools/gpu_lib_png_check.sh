set -o pipefail
# tools/gpu_png_check.sh with the library $LIB (an experiment build) instead of the product
cd $GRAFT_REPO_ROOT; export MMX_LIB_PATH=$GRAFT_REPO_ROOT/$LIB; md5sum $LIB; bash tools/gpu_png_check.sh
