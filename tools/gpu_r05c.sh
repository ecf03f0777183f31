#!/bin/bash
# r05: image statistics kernel + single-pass PNG encoder: GPU tests, bytes A/B against the two-pass
# encoder, dataset kernel trace (collection only) and the 8192-env dataset bench with the writer.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
true ||
true
timeout -k 10 300 python -u tools/png_ab.py > gpurun_out/png_ab_single.json 2> gpurun_out/png_ab_single.err || exit 1
MMX_LIB_PATH=build/libmmx_png2pass.so timeout -k 10 300 python -u tools/png_ab.py > gpurun_out/png_ab_2pass.json 2> gpurun_out/png_ab_2pass.err || exit 1
cat gpurun_out/png_ab_single.json gpurun_out/png_ab_2pass.json
bash tools/gpu_ds_kernels.sh > gpurun_out/ds_kernels.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 \
  --out gpurun_out/ds8192_128.json > gpurun_out/ds8192_128.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 224 \
  --out gpurun_out/ds8192_224.json > gpurun_out/ds8192_224.log 2>&1 || exit 1
grep -h "frames_per_s" gpurun_out/ds8192_128.json gpurun_out/ds8192_224.json gpurun_out/dsk/nowrite.json
