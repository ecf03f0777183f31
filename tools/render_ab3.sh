set -o pipefail
# render-only A/B (tools/render_time.py), interleaved builds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/render_ab3.txt
for r in 1 2; do for v in ${RVARIANTS:-base main}; do
  if [ $v = main ]; then unset MMX_LIB_PATH; else export MMX_LIB_PATH=build/libmmx_$v.so; fi
  timeout -k 10 200 python -u tools/render_time.py > gpurun_out/rt.log 2>&1 || exit 1
  echo "$v $(grep -h '^{' gpurun_out/rt.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["render_ms_mean"],3), [round(p["render_ms"],2) for p in d["points"]])')" >> gpurun_out/render_ab3.txt
done; done
sort gpurun_out/render_ab3.txt
