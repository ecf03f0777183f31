#!/bin/bash
# r05 experiment: does an 11th env per CU pay?  build/libmmx_max40.so (contact cap 40: EnvSh fits 11
# per CU) against itself held at 10 per CU by 1,100 B of dynamic LDS (MMX_LDS_PAD), C3 512-step
# windows, interleaved; plus the product for reference
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/occ11; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2 3; do
  for v in "max40:0" "max40:1100" "product:0"; do
    n=${v%%:*}; pad=${v##*:}
    lib=build/libmmx_max40.so; [ $n = product ] && lib=mujoco_manip_amd/libmmx.so
    MMX_LIB_PATH=$lib MMX_LDS_PAD=$pad timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 512 --warmup 32 \
      --repeats 1 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    echo "$n pad$pad $(grep -h '^{' $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['roofline']['kernel_ms'],3))")" | tee -a $OUT/ab.txt
  done
done
