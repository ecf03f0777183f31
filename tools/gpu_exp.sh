set -o pipefail
# A/B of the product library against an experiment build (MMX_LIB_PATH=$ALT) over a lane sweep
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/exp.txt
ALT=${ALT:-build/libmmx_e192.so}
for lib in mujoco_manip_amd/libmmx.so $ALT; do
for cfg in ${SWEEP:-"4:4096" "2:4096" "1:2048" "1:1536"}; do
  st=${cfg%%:*}; ne=${cfg##*:}
  MMX_LIB_PATH=$lib MMX_STREAMS=$st timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 200 --warmup 30 --envs-per-gpu $ne > gpurun_out/sw.log 2>&1 || exit 1
  echo "$lib streams=$st envs=$ne $(grep -h '^{' gpurun_out/sw.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["solver"]["mean_nefc"])')" >> gpurun_out/exp.txt
done; done
cat gpurun_out/exp.txt
