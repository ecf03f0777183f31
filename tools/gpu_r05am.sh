#!/bin/bash
# r05 end: C5 with the render beside the next step: 128 vs 192 LDS rows, 2 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/c5rows; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for rows in 128 192; do
    MMX_STEP_ROWS=$rows timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "rows$rows $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
  done
done
