#!/bin/bash
# r05: C3 launch shape with the longest-first order: steps per launch (MMX_FUSE) x rollout lanes
# (MMX_STREAMS), 2 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/fuse; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for cfg in ${CFGS:-16,4 8,4 4,4 16,2 8,2 16,1}; do
    f=${cfg%,*}; l=${cfg#*,}
    MMX_FUSE=$f MMX_STREAMS=$l timeout -k 10 300 python -u bench.py --workload ${WL:-c3} --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "fuse$f lanes$l $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
  done
done
