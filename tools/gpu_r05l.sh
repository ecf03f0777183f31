#!/bin/bash
# r05: two env-step kernel layouts in one library (128 rows default without cameras, 192 with):
# full GPU suite with margins, then C5 / C2 / C3 bench lines of the product
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_dual.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_dual.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_dual.log
[ $rc -ne 0 ] && exit $rc
for w in c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_dual_$w.log 2>&1 || exit 1
  MMX_STEP_ROWS=128 timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_dual_${w}_r128.log 2>&1 || exit 1
  MMX_STEP_ROWS=192 timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_dual_${w}_r192.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dual_c3.log 2>&1 || exit 1
for f in gpurun_out/bench_dual_*.log; do echo "$f $(grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), [round(v) for v in d['repeats']['values']])")"; done
