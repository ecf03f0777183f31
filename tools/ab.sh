#!/bin/bash
# Parameterised A/B runner for experiment builds (tools/ab_build.py -> build/libmmx_<name>.so), run on
# the GPU box.  Replaces the r01-r03 one-off gpu_*.sh / render_ab*.sh scripts.
#   LIBS="build/libmmx_a.so build/libmmx_b.so"  builds to compare (the product libmmx.so is always first)
#   ROUNDS=3        interleaved bench rounds (C3 line: --steps STEPS --warmup 32 --repeats 1)
#   STEPS=512       timed env steps per bench run
#   WORKLOAD=c3     bench workload
#   TESTS=0|1       run the GPU parity suite with every library first (stops at the first failure)
#   PMC=0|1         one SQ counter pass per library (VALU, LDS bank conflicts, active lanes)
# Output: gpurun_out/ab/ab.txt (one line per run) and gpurun_out/ab/report.json (tools/ab_report.py).
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out/ab; mkdir -p $OUT; : > $OUT/ab.txt
ALL="mujoco_manip_amd/libmmx.so $LIBS"
if [ "${TESTS:-0}" = 1 ]; then
  for lib in $ALL; do
    n=$(basename $lib .so)
    MMX_LIB_PATH=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/tests_$n.log 2>&1 || { tail -5 $OUT/tests_$n.log; exit 1; }
    echo "$n: $(tail -1 $OUT/tests_$n.log)"
  done
fi
for r in $(seq 1 ${ROUNDS:-3}); do for lib in $ALL; do
  n=$(basename $lib .so)
  MMX_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --workload ${WORKLOAD:-c3} --no-cpu-baseline \
    --steps ${STEPS:-512} --warmup 32 --repeats 1 > $OUT/bench_$n.log 2>&1 || { tail -5 $OUT/bench_$n.log; exit 1; }
  echo "$n $(grep -h '^{' $OUT/bench_$n.log)" >> $OUT/ab.txt
done; done
if [ "${PMC:-0}" = 1 ]; then
  for lib in $ALL; do
    n=$(basename $lib .so)
    (cd /tmp && export TMPDIR=/tmp && MMX_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc \
      SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
      SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/pmc_$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py \
      --workload ${WORKLOAD:-c3} --steps 32 --warmup 32 --repeats 1 --no-cpu-baseline > $OUT/pmc_$n.log 2>&1) \
      || { tail -5 $OUT/pmc_$n.log; exit 1; }
  done
fi
python3 tools/ab_report.py $OUT
