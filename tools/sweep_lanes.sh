set -o pipefail
# rollout-lane / batch-size sweep of the bench (diagnostic); SWEEP overrides the "streams envs" list
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/sweep.txt
for cfg in ${SWEEP:-"1:1024" "1:1280" "1:1536" "1:1792" "2:4096" "4:4096" "8:4096" "3:4608"}; do
  st=${cfg%%:*}; ne=${cfg##*:}
  MMX_STREAMS=$st timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 100 --warmup 30 --envs-per-gpu $ne > gpurun_out/sw.log 2>&1 || exit 1
  echo "streams=$st envs=$ne $(grep -h '^{' gpurun_out/sw.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
