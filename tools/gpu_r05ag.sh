#!/bin/bash
# r05: the driver's configuration (--steps 20 --warmup 5) with the longest-first order vs the launch
# count per rollout call (MMX_MIN_ROUNDS: launches per lane of a call, default 8 -> 3-step launches)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/mr; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2 3; do
  for m in 8 4 6 12 20; do
    MMX_MIN_ROUNDS=$m timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "minrounds$m $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), [round(x) for x in d['repeats']['values']])")" | tee -a $OUT/ab.txt
  done
done
