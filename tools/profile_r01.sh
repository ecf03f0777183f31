#!/bin/bash
# rocprofv3 kernel trace + stats, then separate PMC passes for HBM traffic (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950).  Run on the GPU box from the repo root.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 $ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 $ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_write.log 2>&1
find $OUT -name "*.csv" | head -20
