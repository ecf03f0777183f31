#!/bin/bash
# r05: the order kernel as one wave beside the other lanes' step launches (product) vs 1,024 lanes
# (build/libmmx_o1024.so = the previous commit): C3 A/B, then a kernel trace of the product's C3 run
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="build/libmmx_o1024.so" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/ord_trace; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 64 --repeats 1 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit 1
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -4 $f
