#!/bin/bash
# r05 first GPU call: VALU-issue calibration, GPU suite with recorded parity margins, the 48-episode
# C3 oracle + solver-exit tests on the build without the line-search shortcut, driver-config bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./tools/calib/valu_peak > gpurun_out/valu_peak.json 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/calib_pmc -o run -- $GRAFT_REPO_ROOT/tools/calib/valu_peak \
    > $GRAFT_REPO_ROOT/gpurun_out/calib_pmc.log 2>&1 ) && \
MMX_MARGINS_OUT=gpurun_out/parity_margins.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
MMX_LIB_PATH=build/libmmx_noshortcut.so MMX_MARGINS_OUT=gpurun_out/parity_margins_noshortcut.json \
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pinning.py -q -s --timeout 300 --timeout-method thread \
  -k "c3_episodes_match_oracle or solver_exit_criteria" > gpurun_out/gpu_tests_noshortcut.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver_cfg.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests_noshortcut.log; grep -h "^{" gpurun_out/bench_driver_cfg.log | cut -c1-300; exit $rc
