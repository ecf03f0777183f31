#!/bin/bash
# r05: dataset GPU tests, then 8192-env dataset benches with both step-kernel layouts (interleaved),
# then the 11-envs-per-CU experiment (tools/gpu_r05o.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/dsl; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dataset.py -m gpu -q \
  --timeout 300 --timeout-method thread > $OUT/ds_tests.log 2>&1; rc=$?; tail -2 $OUT/ds_tests.log; [ $rc -ne 0 ] && exit $rc
for args in "128 --no-write" "128" "224"; do
  for rows in 192 128; do
    set -- $args; tag="s$1$( [ -n "$2" ] && echo _nowrite )_r$rows"
    MMX_STEP_ROWS=$rows timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size $args \
      --out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
    echo "$tag $(python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print(round(d['frames_per_s']), d.get('writer_timing'))")"
  done
done
bash tools/gpu_r05o.sh
