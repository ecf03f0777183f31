set -o pipefail
# GPU parity suite, then the bench in the driver's configuration and the default C3 / C2 windows
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/v; : > gpurun_out/v/res.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v/gpu_tests.log 2>&1 || { tail -30 gpurun_out/v/gpu_tests.log; exit 1; }
tail -1 gpurun_out/v/gpu_tests.log >> gpurun_out/v/res.txt
run() { name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/v/$name.log 2>&1 || { tail gpurun_out/v/$name.log; exit 1; }
  echo "$name $(grep -h '^{' gpurun_out/v/$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), [round(v) for v in d["repeats"]["values"]], round(d["roofline"]["kernel_ms"],2), round(d["roofline"]["span_ms_per_launch_round"],2), d["roofline"]["env_steps_per_launch"])')" >> gpurun_out/v/res.txt
}
run driver --steps 20 --warmup 5 && run c3 ${C3ARGS:-} && run c2 --workload c2 --repeats 3
cat gpurun_out/v/res.txt
