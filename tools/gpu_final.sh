set -o pipefail
# round-end call: GPU suite (stop on a failure), then the round evidence (tools/gpu_round_evidence.sh:
# bench lines, rocprof stats + PMC, driver-configuration trace) and the f2 dataset benches
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
md5sum mujoco_manip_amd/*.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -6 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
ROUND=${ROUND:-r04e} DATASET="--num-envs 8192 --episodes 8192 --image-size 128" bash tools/gpu_round_evidence.sh || exit 1
if [ "${DS224:-1}" = 1 ]; then
  timeout -k 10 500 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 224 \
    --out gpurun_out/${ROUND:-r04e}_dataset_bench_224.json > gpurun_out/ds224.log 2>&1 || exit 1
  grep -h frames_per_s gpurun_out/${ROUND:-r04e}_dataset_bench_224.json
fi
