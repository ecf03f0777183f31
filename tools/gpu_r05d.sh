#!/bin/bash
# r05: where the step kernel's waves wait: in-flight levels of VMEM / LDS / SMEM instructions
# (average latency = level / instructions), C3 bench configuration.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
ARGS="--workload c3 --steps 64 --warmup 64 --repeats 1 --no-cpu-baseline"
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INST_LEVEL_VMEM \
    SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv \
    -d $R/gpurun_out/sqlev -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/sqlev.log 2>&1 )
rc=$?; tail -2 gpurun_out/sqlev.log; [ $rc -ne 0 ] && exit $rc
ENVS=8192 SIZE=128 bash tools/gpu_ds_profile.sh
