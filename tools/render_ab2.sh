set -o pipefail
# C5 render A/B: event-timed mmx_render_kernel ms per launch and C5 env steps/s per build, interleaved
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/render_ab.txt
for r in 1 2; do for v in ${RVARIANTS:-base main}; do
  if [ $v = main ]; then unset MMX_LIB_PATH; else export MMX_LIB_PATH=build/libmmx_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/rab.log 2>&1 || exit 1
  echo "$v $(grep -h '^{' gpurun_out/rab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), round(d["render"]["kernel_ms"],3), round(d["roofline"]["kernel_ms"],3))')" >> gpurun_out/render_ab.txt
done; done
sort gpurun_out/render_ab.txt
