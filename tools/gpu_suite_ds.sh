set -o pipefail
# the whole GPU suite and smoke() with the product library, then the 8192-env 224 px dataset bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
md5sum mujoco_manip_amd/libmmx.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 224 \
  --out gpurun_out/ds8192_224.json > gpurun_out/ds8192_224.log 2>&1 || exit 1
grep -h "frames_per_s\|png_mean_bytes" gpurun_out/ds8192_224.json
