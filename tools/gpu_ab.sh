set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
MMX_LIB_PATH=build/libmmx_2w.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_2w.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_2w.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench_main.log 2>&1 && \
MMX_LIB_PATH=build/libmmx_2w.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench_alt.log 2>&1
rc=$?; grep -h "^{" gpurun_out/bench_main.log gpurun_out/bench_alt.log | cut -c100-260; exit $rc
