set -o pipefail
# A/B of several builds (MMX_LIB_PATH) on the C3 bench line, interleaved, 2 rounds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab.txt
for r in 1 2; do for lib in mujoco_manip_amd/libmmx.so $LIBS; do
  MMX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 256 --warmup 32 --repeats 1 > gpurun_out/ab.log 2>&1 || exit 1
  echo "$lib $(grep -h '^{' gpurun_out/ab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["solver"]["mean_nefc"])')" >> gpurun_out/ab.txt
done; done
sort gpurun_out/ab.txt
