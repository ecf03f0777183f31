set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gpu_probe.py digest > gpurun_out/dig_new.log 2>&1 && cp gpurun_out/probe.json gpurun_out/digest_new.json && \
MMX_LIB_PATH=build/libmmx_base.so timeout -k 10 200 python -u tools/gpu_probe.py digest > gpurun_out/dig_base.log 2>&1 && cp gpurun_out/probe.json gpurun_out/digest_base.json && \
python3 -c "
import json; a=json.load(open('gpurun_out/digest_new.json'))['digest']; b=json.load(open('gpurun_out/digest_base.json'))['digest']
print('EPA digests equal:', a['digests']==b['digests'], a['digests'][:3], b['digests'][:3])" && \
LIBS=build/libmmx_base.so ROUNDS=3 STEPS=512 timeout -k 10 600 bash tools/ab.sh > gpurun_out/ab_epa.log 2>&1; tail -4 gpurun_out/ab_epa.log; \
timeout -k 10 900 python -u tools/sweep_env.py --bench-args "--steps 20 --warmup 5" --rounds 2 --out gpurun_out/sweep_driver2.json "" \
 "MMX_PLAN=1,3,3,3,3,3,3,1;2,3,3,3,3,3,2,1;3,3,3,3,3,3,2;3,3,3,3,3,3,1,1" \
 "MMX_PLAN=3,3,3,3,3,3,1,1;1,3,3,3,3,3,3,1;2,3,3,3,3,3,2,1;3,3,3,3,3,2,2,1" \
 "MMX_PLAN=1,3,3,3,3,3,2,1,1;2,3,3,3,3,3,2,1;3,3,3,3,3,3,1,1;3,3,3,3,3,2,2,1" \
 "MMX_PLAN=4,4,4,4,2,1,1;1,4,4,4,4,2,1;2,4,4,4,4,1,1;3,4,4,4,3,1,1" \
 "MMX_PLAN=2,2,2,2,2,2,2,2,2,2;1,2,2,2,2,2,2,2,2,2,1;2,2,2,2,2,2,2,2,2,2;1,2,2,2,2,2,2,2,2,2,1" \
 "MMX_PLAN=5,5,5,3,1,1;1,5,5,5,2,1,1;2,5,5,5,2,1;3,5,5,5,1,1" > gpurun_out/sweep_driver2.log 2>&1 && tail -8 gpurun_out/sweep_driver2.log && \
timeout -k 10 900 python -u tools/sweep_env.py --bench-args "--steps 512 --warmup 64 --repeats 1" --rounds 2 --out gpurun_out/sweep_512.json "" \
 "MMX_PLAN=16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16;4,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,12;8,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,8;12,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,4" "MMX_PLAN=16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,15,1;4,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,11,1;8,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,7,1;12,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,3,1" > gpurun_out/sweep_512.log 2>&1 && tail -4 gpurun_out/sweep_512.log && \
bash tools/gpu.sh fsm
