#!/bin/bash
# Render-kernel time per variant build (diagnostic): rocprofv3 kernel stats of a short C5 bench for
# each MMX_LIB_PATH in $LIBS (main = the product build); averages -> gpurun_out/render_prof.txt
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
: > $ROOT/gpurun_out/render_prof.txt
for lib in ${LIBS:-main}; do
  n=$(basename $lib .so)
  if [ $lib = main ]; then unset MMX_LIB_PATH; else export MMX_LIB_PATH=$ROOT/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/rprof/$n -o run -- \
    python3 $ROOT/bench.py --workload c5 --steps 16 --warmup 4 --repeats 1 --no-cpu-baseline \
    > $ROOT/gpurun_out/rprof_$n.log 2>&1 || exit 1
  echo "$n $(grep -h mmx_render_kernel $ROOT/gpurun_out/rprof/$n/run_kernel_stats.csv | cut -d, -f2,4) $(grep -h '^{' $ROOT/gpurun_out/rprof_$n.log | cut -c100-140)" >> $ROOT/gpurun_out/render_prof.txt
done
cat $ROOT/gpurun_out/render_prof.txt
