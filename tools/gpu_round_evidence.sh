set -o pipefail
# End-of-round evidence in one call: bench lines (tools/gpu_evidence.sh), rocprof stats + PMC of the
# default C3 configuration (tools/profile.sh), and rocprof stats of the driver's configuration
# (--steps 20 --warmup 5) with the bench line of that same traced run
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=${ROUND:-r03}
ROUND=$R bash tools/gpu_evidence.sh || exit 1
timeout -k 10 900 bash tools/profile.sh $R > gpurun_out/profile_${R}.log 2>&1 || { tail -20 gpurun_out/profile_${R}.log; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_driver; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${R}_driver_kernel_stats.csv
grep -h '^{' $OUT/bench_trace.log > gpurun_out/${R}_driver_bench_trace.json
head -3 gpurun_out/${R}_driver_kernel_stats.csv
