#!/bin/bash
# r05: camera rollouts with the render of step k beside the env steps of step k + 1 (default) vs the
# phased schedule (MMX_RENDER_OVERLAP=0): render + dataset GPU tests first, then C5, 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/rov; mkdir -p $OUT; : > $OUT/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_render.py tests/test_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for ov in 1 0; do
    MMX_RENDER_OVERLAP=$ov timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "overlap$ov $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3), round(d['render']['kernel_ms'],3))")" | tee -a $OUT/ab.txt
  done
done
