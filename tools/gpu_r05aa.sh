#!/bin/bash
# r05 experiment: rollout step launches in index order (MMX_STEP_ORDER=0) vs longest-first (
# four FSM cost classes, heaviest first; the product default), C5, C3 and C2, 3 interleaved rounds each
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/ord; mkdir -p $OUT; : > $OUT/ab.txt
for w in ${WORKLOADS:-c5 c3 c2}; do
  for r in 1 2 3; do
    for o in ${MODES:-0 1}; do
      MMX_STEP_ORDER=$o timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      echo "$w order$o $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
    done
  done
done
MMX_MARGINS_OUT=$OUT/margins.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
