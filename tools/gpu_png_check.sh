set -o pipefail
# PNG encoder change check: the PNG / dataset GPU tests, then the f2 kernel profile (collect-only, rocprof
# kernel stats) and the 8192-env dataset bench with writing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
md5sum mujoco_manip_amd/libmmx.so
timeout -k 10 600 python -u -m pytest tests -m gpu -k "png or dataset or render" -q --timeout 300 --timeout-method thread \
  > gpurun_out/png_tests.log 2>&1; rc=$?; tail -3 gpurun_out/png_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ds_kernels.sh || exit 1
timeout -k 10 300 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 \
  --out gpurun_out/ds8192_128.json > gpurun_out/ds8192_128.log 2>&1 || exit 1
grep -h "frames_per_s\|png_mean_bytes" gpurun_out/ds8192_128.json gpurun_out/dsk/nowrite.json
