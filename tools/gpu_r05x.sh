#!/bin/bash
# r05 experiment: C5 with the render launched per lane after its step (default) vs one render of all
# envs after every lane's step (MMX_RENDER_PHASED=1), 3 interleaved rounds, 3 windows each
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/rph; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2 3; do
  for ph in 0 1; do
    MMX_RENDER_PHASED=$ph timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "phased$ph $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
  done
done
MMX_RENDER_PHASED=1 timeout -k 10 300 python -u -m pytest tests/test_render.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
