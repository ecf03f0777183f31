set -o pipefail
# round evidence on the GPU box: parity suite, default bench line (C3 + CPU baseline), C2 / C5 lines,
# 2-rank rehearsal on one GPU, rocprofv3 trace + PMC passes (tools/profile.sh); every GPU step under
# its own time limit.  Condense the PMC CSVs on the host afterwards (tools/pmc_traffic.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=${ROUND:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --steps 128 --warmup 32 > gpurun_out/bench_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --share-device --dist-backend gloo --steps 64 --repeats 1 \
   --no-cpu-baseline > gpurun_out/bench_2rank_rehearsal.log 2>&1 && \
bash tools/profile.sh $R > gpurun_out/profile.log 2>&1 && \
WORKLOAD=c5 PROF_STEPS=32 PROF_WARMUP=16 bash tools/profile.sh $R > gpurun_out/profile_c5.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log; for f in bench bench_c2 bench_c5; do grep -h "^{" gpurun_out/$f.log | cut -c1-200; done
exit $rc
