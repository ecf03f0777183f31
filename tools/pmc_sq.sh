#!/bin/bash
# Diagnostic PMC passes (shader sequencer) over a short bench run; one pass per counter set.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- \
    python3 $ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
