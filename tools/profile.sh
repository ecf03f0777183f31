#!/bin/bash
# rocprofv3 evidence for bench.py's default C3 configuration (run on the GPU box from the repo root):
#   1. kernel trace + stats of a bench run                 -> gpurun_out/prof/trace
#   2. separate PMC passes (no trace domains combined with --pmc), same command each:
#        FETCH_SIZE | WRITE_SIZE | 8 SQ counters (VALU issue, LDS, waits)
#   3. tools/pmc_traffic.py condenses them into profiles/<round>_* and profiles/pmc_<workload>.json
#      (per env step, tagged with the configuration; bench.py uses it only for a matching line)
set -e
ROUND=${1:-r03}
WL=${WORKLOAD:-c3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$WL
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=${PROF_STEPS:-64}   # multiples of the 16-step fused launch: equal-size dispatches
WARM=${PROF_WARMUP:-64}
ARGS="--workload $WL --steps $STEPS --warmup $WARM --repeats 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d $OUT/sq -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_sq.log 2>&1
# lane utilisation: thread-cycles of VALU work / (VALU instruction cycles x 64 lanes)
timeout -s KILL 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/lanes -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_lanes.log 2>&1
# extended SQ passes: any-instruction issue, SALU / LDS / branch / memory instruction mix per wave
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sqx_a -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_sqx_a.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU \
  SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sqx_b -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/bench_sqx_b.log 2>&1
cd $ROOT
python3 tools/pmc_traffic.py --round $ROUND --workload $WL --prof $OUT --timed-steps $STEPS
