#!/bin/bash
# r05: C5 with the render of step k beside step k + 1 (MMX_RENDER_OVERLAP=1, poses double-buffered)
# vs the serial phased rollout: bit-identity test, 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/rov; mkdir -p $OUT; : > $OUT/ab.txt
timeout -k 10 300 python -u -m pytest tests/test_render.py -m gpu -x -q -k "overlap or c5_full" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for o in 0 1; do
    MMX_RENDER_OVERLAP=$o timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "overlap$o $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3), round(d['render']['kernel_ms'],3), round(d['roofline']['kernel_ms'],3))")" | tee -a $OUT/ab.txt
  done
done
