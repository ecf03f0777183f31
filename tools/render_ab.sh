set -o pipefail
# C5 render cost split (diagnostic): baseline vs builds that skip raster / shading stages
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/render_ab.txt
for v in ${RVARIANTS:-main rs1}; do
  if [ $v = main ]; then unset MMX_LIB_PATH; else export MMX_LIB_PATH=build/libmmx_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/rab.log 2>&1 || exit 1
  echo "$v $(grep -h '^{' gpurun_out/rab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')" >> gpurun_out/render_ab.txt
done
cat gpurun_out/render_ab.txt
