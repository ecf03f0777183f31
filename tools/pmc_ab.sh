#!/bin/bash
# PMC A/B: one SQ counter pass per library (MMX_LIB_PATH) over a short C3 bench; raw CSVs under
# gpurun_out/pmc_ab/<name>/ (condensed on the host).  Diagnostic.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  name=$(basename $lib .so)
  MMX_LIB_PATH=$ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv \
    -d $ROOT/gpurun_out/pmc_ab/$name -o run -- python3 $ROOT/bench.py --steps 32 --warmup 32 --repeats 1 \
    --no-cpu-baseline > $ROOT/gpurun_out/pmc_ab_$name.log 2>&1
done
