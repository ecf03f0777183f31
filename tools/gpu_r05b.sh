#!/bin/bash
# r05 second GPU call: scalar / packed VALU calibration (+ SQ counters of the scalar one), the smooth
# dynamics known answers on the kernel, extended SQ counter passes of the C3 step kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/calib/valu_peak > gpurun_out/valu_peak_scalar.json 2>&1 && \
timeout -k 10 60 ./tools/calib/valu_peak_pk > gpurun_out/valu_peak_packed.json 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/calib_pmc_scalar -o run -- $R/tools/calib/valu_peak \
    > $R/gpurun_out/calib_pmc_scalar.log 2>&1 ) && \
MMX_MARGINS_OUT=gpurun_out/parity_margins_smooth.json timeout -k 10 300 python -u -m pytest tests/test_smooth_dynamics_kat.py \
  -q -s --timeout 120 --timeout-method thread > gpurun_out/gpu_smooth.log 2>&1 ; \
ARGS="--workload c3 --steps 64 --warmup 64 --repeats 1 --no-cpu-baseline"
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/sqx_a -o run -- \
    python3 $R/bench.py $ARGS > $R/gpurun_out/sqx_a.log 2>&1 ) && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
    SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv \
    -d $R/gpurun_out/sqx_b -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/sqx_b.log 2>&1 )
rc=$?; tail -3 gpurun_out/gpu_smooth.log; head -3 gpurun_out/valu_peak_scalar.json; exit $rc
