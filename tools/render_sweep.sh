#!/bin/bash
# Renderer A/B (diagnostics): isolated render time (tools/render_time.py) and one SQ pass (LDS bank
# conflicts) of mmx_render_kernel per library.  LIBS="build/libmmx_x.so ..."; the product first.
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/rsweep; mkdir -p $OUT; : > $OUT/times.txt
for lib in mujoco_manip_amd/libmmx.so $LIBS; do
  n=$(basename $lib .so)
  MMX_LIB_PATH=$lib timeout -k 10 300 python -u tools/render_time.py --reps 10 > $OUT/time_$n.json 2> $OUT/time_$n.err || exit 1
  echo "$n $(python3 -c "import json;print(round(json.load(open('$OUT/time_$n.json'))['render_ms_mean'],4))")" >> $OUT/times.txt
  (cd /tmp && export TMPDIR=/tmp && MMX_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -s KILL 200 rocprofv3 \
    --kernel-include-regex mmx_render_kernel --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_INSTS_LDS SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_$n -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/render_time.py --reps 2 > $GRAFT_REPO_ROOT/$OUT/pmc_$n.log 2>&1) || exit 1
done
cat $OUT/times.txt
