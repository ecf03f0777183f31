set -o pipefail
# occupancy probe: envs (one resident round = 2048 at 8 per CU) x rollout lanes, fused launches
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/occ.txt
for cfg in ${SWEEP:-"1:2048" "2:2048" "4:2048" "1:1024" "4:1024" "1:4096" "4:4096" "8:4096"}; do
  st=${cfg%%:*}; ne=${cfg##*:}
  MMX_STREAMS=$st timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 256 --warmup 32 --envs-per-gpu $ne > gpurun_out/oc.log 2>&1 || exit 1
  echo "streams=$st envs=$ne $(grep -h '^{' gpurun_out/oc.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["solver"]["mean_nefc"])')" >> gpurun_out/occ.txt
done
cat gpurun_out/occ.txt
