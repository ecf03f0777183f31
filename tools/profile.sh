#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of a short bench run      -> gpurun_out/prof/trace/*kernel_stats.csv
#   2. separate PMC passes for FETCH_SIZE, WRITE_SIZE  -> gpurun_out/prof/{fetch,write}/*counter_collection.csv
#      (gfx950: the two counters cannot share a pass; no trace domains combined with --pmc)
#   3. tools/pmc_traffic.py condenses them into profiles/<round>_* and profiles/pmc_traffic.json
set -e
ROUND=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=${PROF_STEPS:-48}  # multiples of the 16-step fused launch: equal-size dispatches
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOT/bench.py --steps $STEPS --warmup 16 --no-cpu-baseline > $OUT/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $ROOT/bench.py --steps 16 --warmup 16 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $ROOT/bench.py --steps 16 --warmup 16 --no-cpu-baseline > $OUT/bench_write.log 2>&1
cd $ROOT
python3 tools/pmc_traffic.py --round $ROUND --prof $OUT
