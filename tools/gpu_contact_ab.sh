set -o pipefail
# contact-list A/B: $BASE vs the working tree on the same states (tools/contact_ab.py)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BASE=${BASE:-build/libmmx_base.so}
MMX_LIB_PATH=$BASE timeout -k 10 200 python -u tools/contact_ab.py gen > gpurun_out/cab_gen.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/contact_ab.py cmp > gpurun_out/cab_cmp.log 2>&1 || exit 1
cat gpurun_out/cab_cmp.log
