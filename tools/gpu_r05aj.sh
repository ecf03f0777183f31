#!/bin/bash
# r05: the class-major, rows-minor order as the product: GPU tests (order bit-identity, rollouts,
# render), C5 and C3 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/ordr; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_render.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $OUT/c5.log 2>&1 || exit 1
grep -h '^{' $OUT/c5.log > $OUT/r05_bench_c5.json
timeout -k 10 400 python -u bench.py > $OUT/c3.log 2>&1 || exit 1
grep -h '^{' $OUT/c3.log > $OUT/r05_bench_c3.json
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drv.log 2>&1 || exit 1
grep -h '^{' $OUT/drv.log > $OUT/r05_bench_driver_cfg.json
for f in $OUT/r05_bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), [round(x) for x in d['repeats']['values']])"; done
