cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/c2sweep.txt
for cfg in "1:1" "1:16" "2:16" "4:16" "4:4" "2:4"; do
  st=${cfg%%:*}; fu=${cfg##*:}
  MMX_STREAMS=$st MMX_FUSE=$fu timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/c2s.log 2>&1 || exit 1
  echo "C2 streams=$st fuse=$fu $(grep -h '^{' gpurun_out/c2s.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')" >> gpurun_out/c2sweep.txt
done
cat gpurun_out/c2sweep.txt
