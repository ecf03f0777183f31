set -o pipefail
# Sweep of env steps per launch (MMX_FUSE) x rollout lanes (MMX_STREAMS) on the C3 bench line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/fuse.txt
for cfg in ${SWEEP:-"4:1" "4:8" "4:32" "4:100" "1:32" "2:32"}; do
  st=${cfg%%:*}; fu=${cfg##*:}
  MMX_STREAMS=$st MMX_FUSE=$fu timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fs.log 2>&1 || exit 1
  echo "streams=$st fuse=$fu $(grep -h '^{' gpurun_out/fs.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],3), round(r["kernel_ms"],2), d["solver"]["mean_nefc"])')" >> gpurun_out/fuse.txt
done
cat gpurun_out/fuse.txt
