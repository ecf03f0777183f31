set -o pipefail
# GPU suite on the working-tree build, then per-FSM-state phase profiles (diagnostic builds) and
# an interleaved bench A/B of $BASE (default build/libmmx_base.so) against the working tree.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -4 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
BASEP=${BASEP:-build/libmmx_basep.so}
BASE=${BASE:-build/libmmx_base.so}
MMX_PROFILE=1 MMX_LIB_PATH=$BASEP timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_base.log 2>&1 || exit 1
cp gpurun_out/probe_prof.json gpurun_out/fsm_base.json
MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_new.log 2>&1 || exit 1
cp gpurun_out/probe_prof.json gpurun_out/fsm_new.json
: > gpurun_out/ab.txt
for r in 1 2; do for lib in $BASE mujoco_manip_amd/libmmx.so; do
  MMX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 512 --warmup 64 --repeats 1 > gpurun_out/ab.log 2>&1 || exit 1
  echo "$lib $(grep -h '^{' gpurun_out/ab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["solver"]["mean_nefc"])')" >> gpurun_out/ab.txt
done; done
cat gpurun_out/ab.txt
