set -o pipefail
# launch-shape experiment 3: small launches in the driver config and in 512-step windows
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fuse; : > gpurun_out/fuse/res3.txt
run() { # steps warmup repeats fuse streams
  MMX_STREAMS=$5 MMX_FUSE=$4 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps $1 --warmup $2 --repeats $3 > gpurun_out/fuse/e.log 2>&1 || { tail gpurun_out/fuse/e.log; exit 1; }
  echo "steps=$1 fuse=$4 streams=$5 $(grep -h '^{' gpurun_out/fuse/e.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), [round(v) for v in d["repeats"]["values"]], round(d["roofline"]["kernel_ms"],2), round(d["roofline"]["span_ms_per_launch_round"],2))')" >> gpurun_out/fuse/res3.txt
}
run 20 5 5 4 4 && run 20 5 5 3 4 && run 20 5 5 2 4 && run 20 5 5 5 8 && run 20 5 5 5 3 && \
run 512 64 2 16 4 && run 512 64 2 8 4 && run 512 64 2 4 4 && run 512 64 2 2 4 && run 20 5 5 16 4
cat gpurun_out/fuse/res3.txt
