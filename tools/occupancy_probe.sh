#!/bin/bash
# Occupancy sensitivity of the step kernel (diagnostics): C3 env steps/s at 8 / 7 / 6 / 5 / 4
# envs per CU (extra dynamic LDS per workgroup, MMX_LDS_PAD) for the product build, and the
# product against the 168-VGPR build (MMX_STEP_WAVES=3) at the product's 8 per CU, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/occ
A="--steps 128 --warmup 32 --repeats 3 --no-cpu-baseline"
for rep in 1 2; do
  for pad in 0 2096 6192 12336 20528; do
    MMX_LDS_PAD=$pad timeout -k 10 200 python -u bench.py $A > gpurun_out/occ/pad${pad}_$rep.log 2>&1 || exit 1
  done
  MMX_LIB_PATH=build/libmmx_w3.so timeout -k 10 200 python -u bench.py $A > gpurun_out/occ/w3_$rep.log 2>&1 || exit 1
done
for f in gpurun_out/occ/*.log; do echo -n "$f "; grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), [round(v) for v in d['repeats']['values']])"; done
