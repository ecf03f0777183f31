#!/bin/bash
# r05 evidence of the 11-per-CU product: rocprof stats + PMC + extended SQ of C3 (tools/profile.sh),
# bench lines C3 (with the CPU baseline) / driver config / C2 / C5 (tools/gpu_evidence.sh), the
# 8192-env dataset benches, the per-FSM-phase profile; box-side profiles copied under gpurun_out/box_profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/box_profiles
timeout -k 10 900 bash tools/profile.sh r05 > gpurun_out/profile_r05.log 2>&1 || { tail -20 gpurun_out/profile_r05.log; exit 1; }
cp profiles/r05_c3_* profiles/pmc_c3.json gpurun_out/box_profiles/ || exit 1
ROUND=r05 bash tools/gpu_evidence.sh || exit 1
for a in "128 --no-write" "128" "224"; do
  set -- $a; tag="ds_s$1$( [ -n "$2" ] && echo _nowrite )"
  timeout -k 10 400 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size $a \
    --out gpurun_out/$tag.json > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
  echo "$tag $(python3 -c "import json; print(round(json.load(open('gpurun_out/$tag.json'))['frames_per_s']))")"
done
MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm_default.log 2>&1 || { tail -5 gpurun_out/fsm_default.log; exit 1; }
cp gpurun_out/probe_prof.json gpurun_out/fsm_default.json
