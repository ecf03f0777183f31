#!/bin/bash
# r05 end: C5 with the render stream at default / lowest / highest priority, 2 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/prio; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for p in 0 -1 1; do
    MMX_RSTREAM_PRIO=$p timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "prio$p $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
  done
done
