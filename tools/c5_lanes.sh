cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/c5lanes.txt
for st in 8 4 2; do
  MMX_STREAMS=$st timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --steps 128 --warmup 16 > gpurun_out/c5l.log 2>&1 || exit 1
  echo "C5 streams=$st $(grep -h '^{' gpurun_out/c5l.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')" >> gpurun_out/c5lanes.txt
done
cat gpurun_out/c5lanes.txt
