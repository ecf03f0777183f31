set -o pipefail
# full GPU parity suite (one pytest process), then a short C3 bench; logs under gpurun_out/
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log | grep -E "PASS|FAIL|ERROR|passed|failed|Error" | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 256 > gpurun_out/bench_quick.log 2>&1
rc=$?; grep -h "^{" gpurun_out/bench_quick.log | cut -c1-300; exit $rc
