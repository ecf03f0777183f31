#!/bin/bash
# r05: dataset path with per-slot PNG buffers (mmx_copy_ranges): dataset GPU tests, 8192-env benches
# (128^2 with / without the writer + cProfile, 224^2 with the writer), collection-only with the
# 128-row step kernel for the layout comparison
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dataset.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/ds_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ds_tests.log; [ $rc -ne 0 ] && exit $rc
ENVS=8192 SIZE=128 bash tools/gpu_ds_profile.sh || exit 1
timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 224 \
  --out gpurun_out/ds8192_224.json > gpurun_out/ds8192_224.log 2>&1 || exit 1
MMX_STEP_ROWS=128 timeout -k 10 300 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 \
  --no-write --out gpurun_out/ds_nowrite_r128.json > gpurun_out/ds_nowrite_r128.log 2>&1 || exit 1
grep -h "frames_per_s" gpurun_out/ds8192_224.json gpurun_out/ds_nowrite_r128.json
