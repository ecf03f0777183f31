#!/bin/bash
# r05: camera rollouts on one lane (one longest-first step launch + one render per step): render +
# rollout GPU tests, C5 bench line, render SQ counters of the new launch shape
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/c5l1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_render.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b$r.log 2>&1 || { tail -5 $OUT/b$r.log; exit 1; }
  grep -h '^{' $OUT/b$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['value']), round(d['ms_per_step'],3), d['render']['kernel_ms'], d['roofline']['achieved'])"
done
bash tools/render_pmc.sh && python3 tools/render_pmc.py --round r05 > $OUT/rpmc.txt && cp profiles/r05_render_pmc.json $OUT/ && tail -12 $OUT/rpmc.txt
