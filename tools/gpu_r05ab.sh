#!/bin/bash
# r05: dataset collection with the env steps in index order (MMX_STEP_ORDER=0) vs longest first
# (default), 8192 envs x 8192 episodes at 128^2 without the writer, 2 interleaved rounds; dataset tests
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/dso; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for o in 0 1; do
    tag="o${o}_r$r"
    MMX_STEP_ORDER=$o timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 --no-write \
      --out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
    echo "order$o $(python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print(round(d['frames_per_s']))")" | tee -a $OUT/ab.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_dataset.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/ds_tests.log 2>&1; tail -2 $OUT/ds_tests.log
