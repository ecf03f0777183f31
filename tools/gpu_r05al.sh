#!/bin/bash
# r05 end: camera rollouts with the render beside the next step by default: GPU suite (margins),
# smoke(), C5 bench line, C5 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_end.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_end.log 2>&1; rc=$?; tail -1 gpurun_out/gpu_tests_end.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1 || { tail -5 gpurun_out/smoke_end.log; exit 1; }
tail -1 gpurun_out/smoke_end.log
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05_bench_c5.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r05_bench_c5.log > gpurun_out/r05_bench_c5.json
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_c5.json')); print(round(d['value']), [round(x) for x in d['repeats']['values']], d['roofline']['kernel_ms'], d['render']['kernel_ms'], d['render']['isolated'])"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_c5; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --no-cpu-baseline --steps 64 --warmup 16 --repeats 1 > $OUT/bench_trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r05_c5_kernel_stats.csv
grep -h '^{' $OUT/bench_trace.log > gpurun_out/r05_c5_bench_trace.json
head -4 gpurun_out/r05_c5_kernel_stats.csv
