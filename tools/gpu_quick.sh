set -o pipefail
# parity suite + a short bench (no CPU baseline): the edit-measure loop on the GPU box
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench_quick.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; grep -h "^{" gpurun_out/bench_quick.log | cut -c1-400; exit $rc
