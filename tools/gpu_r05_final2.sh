#!/bin/bash
# r05 end, part 2: 8192-env dataset benches, the per-FSM-phase profile, C5 rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for a in "128 --no-write" "128" "224"; do
  set -- $a; tag="ds_s$1$( [ -n "$2" ] && echo _nowrite )"
  timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size $a \
    --out gpurun_out/$tag.json > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
  echo "$tag $(python3 -c "import json; print(round(json.load(open('gpurun_out/$tag.json'))['frames_per_s']))")"
done
MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_default.log 2>&1 || { tail -5 gpurun_out/fsm_default.log; exit 1; }
cp gpurun_out/probe_prof.json gpurun_out/fsm_default.json
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_c5; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --no-cpu-baseline --steps 64 --warmup 16 --repeats 1 > $OUT/bench_trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r05_c5_kernel_stats.csv
grep -h '^{' $OUT/bench_trace.log > gpurun_out/r05_c5_bench_trace.json
echo final2 done
