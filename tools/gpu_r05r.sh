#!/bin/bash
# r05: with the 128-row kernel at 11 envs per CU, which layout wins per workload? C5 / C2 bench lines
# and the 8192-env dataset collection with MMX_STEP_ROWS=128 vs 192, two interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/lay; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for w in c5 c2; do
    for rows in 128 192; do
      timeout -k 10 300 python -u bench.py --workload $w --step-rows $rows --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      echo "$w r$rows $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']))")" | tee -a $OUT/ab.txt
    done
  done
  for rows in 128 192; do
    MMX_STEP_ROWS=$rows timeout -k 10 300 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 \
      --no-write --out $OUT/ds.json > $OUT/ds.log 2>&1 || { tail -5 $OUT/ds.log; exit 1; }
    echo "ds_collect r$rows $(python3 -c "import json; print(round(json.load(open('$OUT/ds.json'))['frames_per_s']))")" | tee -a $OUT/ab.txt
  done
done
