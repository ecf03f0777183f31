#!/bin/bash
# r05: C5 with the order: one lane + one render per step (product) vs a render per lane after its
# own step (MMX_RENDER_PHASED=0) on 2 / 4 lanes, 2 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/c5ph; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for cfg in "1 4" "0 2" "0 4" "0 3"; do
    set -- $cfg
    MMX_RENDER_PHASED=$1 MMX_STREAMS=$2 timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --repeats 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "phased$1 streams$2 $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))")" | tee -a $OUT/ab.txt
  done
done
