#!/bin/bash
# r05: cross-lane primitive latencies; dataset GPU tests + host-path profile after the flat scatter
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./tools/calib/prim_lat > gpurun_out/prim_lat.json 2>&1 || exit 1
cat gpurun_out/prim_lat.json
timeout -k 10 600 python -u -m pytest tests/test_dataset.py -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/ds_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ds_tests.log; [ $rc -ne 0 ] && exit $rc
ENVS=8192 SIZE=128 bash tools/gpu_ds_profile.sh
