set -o pipefail
# Round evidence: bench lines (C3 with the CPU baseline, the driver's short config, C2, C5) and an
# f2 dataset-generation throughput run; outputs under gpurun_out/ (copied to profiles/ by hand).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=${ROUND:-r03}
timeout -k 10 400 python -u bench.py > gpurun_out/${R}_bench_c3.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${R}_bench_c3.log > gpurun_out/${R}_bench_c3.json
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_bench_driver_cfg.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${R}_bench_driver_cfg.log > gpurun_out/${R}_bench_driver_cfg.json
timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/${R}_bench_c2.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${R}_bench_c2.log > gpurun_out/${R}_bench_c2.json
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/${R}_bench_c5.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${R}_bench_c5.log > gpurun_out/${R}_bench_c5.json
if [ -n "$DATASET" ]; then
  timeout -k 10 500 python -u tools/dataset_bench.py $DATASET --out gpurun_out/${R}_dataset_bench.json > gpurun_out/${R}_dataset_bench.log 2>&1 || exit 1
fi
for f in gpurun_out/${R}_bench_*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'], (d.get('render') or {}).get('kernel_ms'))"; done
