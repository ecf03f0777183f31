#!/bin/bash
# r05: 128 LDS rows / 10 envs per CU: GPU suite (margins), A/B against 192 rows (8 per CU) and 128 rows
# at 8 per CU, driver-config bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_MARGINS_OUT=gpurun_out/parity_margins_l128.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_l128.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_l128.log
[ $rc -ne 0 ] && exit $rc
LIBS="build/libmmx_l192.so build/libmmx_l128w2.so build/libmmx_dovf0.so" ROUNDS=3 bash tools/ab.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver_l128.log 2>&1 || exit 1
grep -h '^{' gpurun_out/bench_driver_l128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver cfg', round(d['value']), [round(v) for v in d['repeats']['values']])"
