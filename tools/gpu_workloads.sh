set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/c5prof
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --steps 200 > gpurun_out/bench_c5.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c5prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --no-cpu-baseline --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/c5prof/bench.log 2>&1
echo done $?
