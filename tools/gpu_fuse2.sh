set -o pipefail
# launch-shape experiment 2 (balanced launch lengths): driver-config windows for MMX_FUSE / MMX_STREAMS
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fuse; : > gpurun_out/fuse/res2.txt
for cfg in 16:4 8:4 7:4 5:4 10:2 16:2 20:1 10:1; do f=${cfg%%:*}; s=${cfg##*:}
  MMX_STREAMS=$s MMX_FUSE=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/fuse/e.log 2>&1 || { tail gpurun_out/fuse/e.log; exit 1; }
  echo "driver fuse=$f streams=$s $(grep -h '^{' gpurun_out/fuse/e.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), [round(v) for v in d["repeats"]["values"]], round(d["roofline"]["kernel_ms"],2), round(d["roofline"]["span_ms_per_launch_round"],2))')" >> gpurun_out/fuse/res2.txt
done
cat gpurun_out/fuse/res2.txt
