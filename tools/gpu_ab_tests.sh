set -o pipefail
# GPU parity suite on the product build, then an interleaved C3 A/B of the product against the
# experiment builds in $LIBS (3 rounds, 512 timed env steps each); results in gpurun_out/ab.txt
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
for r in 1 2 3; do for lib in mujoco_manip_amd/libmmx.so $LIBS; do
  MMX_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 512 --warmup 32 --repeats 1 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/ab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4), round(d["solver"]["mean_nefc"],2), round(d["solver"]["mean_solver_iter"],4))')" >> gpurun_out/ab.txt
done; done
sort gpurun_out/ab.txt
