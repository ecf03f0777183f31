#!/bin/bash
# SQ counters of mmx_render_kernel alone (C5 bench, short): two PMC passes of <= 8 SQ counters each,
# no trace domains combined with --pmc.  Output: gpurun_out/rpmc/{a,b}; condensed by
# tools/render_pmc.py into profiles/<round>_render_pmc.json.  Diagnostic.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="--workload c5 --steps 16 --warmup 4 --repeats 1 --no-cpu-baseline"
rm -rf $ROOT/gpurun_out/rpmc; mkdir -p $ROOT/gpurun_out/rpmc
timeout -s KILL 200 rocprofv3 --kernel-include-regex mmx_render_kernel --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv \
  -d $ROOT/gpurun_out/rpmc/a -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/gpurun_out/rpmc/a.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-include-regex mmx_render_kernel --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv \
  -d $ROOT/gpurun_out/rpmc/b -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/gpurun_out/rpmc/b.log 2>&1 || exit 1
echo render pmc done
