#!/bin/bash
# The one GPU-box runner (replaces the per-experiment gpu_*.sh scripts of r01-r05).  Usage, from the
# repo root on the GPU box (gpurun -- 'bash tools/gpu.sh RECIPE [RECIPE ...]'); recipes run in order and
# the first failure ends the call.  Outputs under gpurun_out/ (copied to profiles/ by hand; the condensed
# PMC files also under gpurun_out/profiles_out/).
#   tests            GPU suite (pytest -m gpu, every failure listed) + smoke()
#   quick            GPU suite (-x) + a 200-step C3 bench line
#   bench:WL         bench line of workload WL (c3 with the CPU baseline; c2, c5; driver = the driver's
#                    --steps 20 --warmup 5 C3 configuration)            -> gpurun_out/$R_bench_WL.json
#   evidence         bench:c3 bench:driver bench:c2 bench:c5
#   profile:WL       rocprofv3 kernel trace + stats and the PMC passes (FETCH, WRITE, SQ, lanes, extended
#                    SQ) of a short WL bench, condensed by tools/pmc_traffic.py
#   trace:driver     rocprofv3 kernel trace of the driver configuration + that run's own line
#   render_pmc       SQ counters of the render kernel (C5)
#   fsm              per-FSM-phase cycle profile (libmmx_prof.so); PROBE_SETS="1 5 ..." adds the
#                    sub-phase probe builds build/libmmx_prof<P>.so (tools/build_probes.py)
#   dataset:S        f2 dataset collection + LeRobot writer, 8192 envs x 8192 episodes, S px
#   ab               interleaved A/B of $LIBS against the product (tools/ab.sh; ROUNDS, STEPS, PMC, TESTS)
#   occupancy        C3 env steps/s with the envs per CU lowered by dynamic LDS per workgroup (MMX_LDS_PAD;
#                    1,280-byte blocks, profiles/r05_lds_residency.json: 12,640 B = 12 per CU; pads 2560 /
#                    6400 / 8960 / 20480 B -> 10 / 8 / 7 / 4 per CU)
# Env: R (round tag, default r06), MMX_LIB_PATH (a library other than the product for every recipe).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; ROOT=$(pwd); mkdir -p gpurun_out
R=${R:-r06}

line() { grep -h '^{' "$1"; }

bench() {  # bench WL
  local wl=$1 args
  case $wl in
    c3) args="" ;;
    driver) args="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" ;;
    c2|c5) args="--workload $wl --no-cpu-baseline" ;;
    *) echo "unknown workload $wl"; return 2 ;;
  esac
  timeout -k 10 400 python -u bench.py $args > gpurun_out/${R}_bench_$wl.log 2>&1 || { tail -5 gpurun_out/${R}_bench_$wl.log; return 1; }
  line gpurun_out/${R}_bench_$wl.log > gpurun_out/${R}_bench_$wl.json
  python3 -c "import json; d=json.load(open('gpurun_out/${R}_bench_$wl.json')); print('$wl', round(d['value']), [round(v) for v in d['repeats']['values']], round(d['roofline']['kernel_ms'], 3), round(d['roofline']['frac'], 3))"
}

profile() {  # profile WL: trace + separate PMC passes (no trace domain combined with --pmc)
  local wl=$1 out=$ROOT/gpurun_out/prof_$1 steps=${PROF_STEPS:-64} warm=${PROF_WARMUP:-64}
  local args="--workload $wl --steps $steps --warmup $warm --repeats 1 --no-cpu-baseline"
  rm -rf $out; mkdir -p $out
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_trace.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_fetch.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_write.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
     SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d $out/sq -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_sq.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $out/lanes -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_lanes.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH \
     SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $out/sqx_a -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_sqx_a.log 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU \
     SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv -d $out/sqx_b -o run -- \
     python3 $ROOT/bench.py $args > $out/bench_sqx_b.log 2>&1) || { tail -5 $out/*.log; return 1; }
  python3 tools/pmc_traffic.py --round $R --workload $wl --prof $out --timed-steps $steps || return 1
  mkdir -p gpurun_out/profiles_out && cp profiles/${R}_${wl}_* profiles/pmc_${wl}.json gpurun_out/profiles_out/  # (only gpurun_out/ comes back)
}

trace_driver() {
  local out=$ROOT/gpurun_out/prof_driver
  rm -rf $out; mkdir -p $out
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace \
     -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_trace.log 2>&1) || return 1
  cp $(find $out/trace -name "*kernel_stats.csv" | head -1) gpurun_out/${R}_driver_kernel_stats.csv
  cp $(find $out/trace -name "*kernel_trace.csv" | head -1) gpurun_out/${R}_driver_kernel_trace.csv
  line $out/bench_trace.log > gpurun_out/${R}_driver_bench_trace.json
}

render_pmc() {
  local args="--workload c5 --steps 16 --warmup 4 --repeats 1 --no-cpu-baseline"
  rm -rf $ROOT/gpurun_out/rpmc; mkdir -p $ROOT/gpurun_out/rpmc
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -s KILL 200 rocprofv3 --kernel-include-regex mmx_render_kernel --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES \
     SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv \
     -d $ROOT/gpurun_out/rpmc/a -o run -- python3 $ROOT/bench.py $args > $ROOT/gpurun_out/rpmc/a.log 2>&1 &&
   timeout -s KILL 200 rocprofv3 --kernel-include-regex mmx_render_kernel --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS \
     SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv \
     -d $ROOT/gpurun_out/rpmc/b -o run -- python3 $ROOT/bench.py $args > $ROOT/gpurun_out/rpmc/b.log 2>&1) || return 1
  python3 tools/render_pmc.py --round $R --prof $ROOT/gpurun_out/rpmc || return 1
  mkdir -p gpurun_out/profiles_out && cp profiles/${R}_render_pmc.json profiles/pmc_render.json gpurun_out/profiles_out/
}

fsm() {
  MMX_PROFILE=1 timeout -k 10 300 python -u tools/gpu_probe.py fsm > gpurun_out/fsm.log 2>&1 || { tail -5 gpurun_out/fsm.log; return 1; }
  cp gpurun_out/probe_prof.json gpurun_out/${R}_fsm_profile.json
  for P in $PROBE_SETS; do
    MMX_PROFILE=1 MMX_LIB_PATH=build/libmmx_prof$P.so timeout -k 10 300 python -u tools/gpu_probe.py fsm \
      > gpurun_out/fsm_set$P.log 2>&1 || { tail -5 gpurun_out/fsm_set$P.log; return 1; }
    cp gpurun_out/probe_prof.json gpurun_out/${R}_fsm_probe_set$P.json
  done
}

tests() {
  md5sum mujoco_manip_amd/*.so
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  local rc=$?; tail -6 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && return $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || return 1
  tail -1 gpurun_out/smoke.log
}

quick() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  local rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && return $rc
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench_quick.log 2>&1 || return 1
  line gpurun_out/bench_quick.log | cut -c1-400
}

dataset() {
  timeout -k 10 500 python -u tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size $1 \
    --out gpurun_out/${R}_dataset_bench_$1.json > gpurun_out/${R}_dataset_$1.log 2>&1 || { tail -5 gpurun_out/${R}_dataset_$1.log; return 1; }
  grep -h "frames_per_s" gpurun_out/${R}_dataset_bench_$1.json
}

occupancy() {
  mkdir -p gpurun_out/occ
  local a="--steps 128 --warmup 32 --repeats 3 --no-cpu-baseline"
  for pad in 0 2560 6400 8960 20480; do
    MMX_LDS_PAD=$pad timeout -k 10 200 python -u bench.py $a > gpurun_out/occ/pad$pad.log 2>&1 || return 1
    echo "pad $pad $(line gpurun_out/occ/pad$pad.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']))")"
  done
}

for recipe in "$@"; do
  echo "== $recipe"
  case $recipe in
    tests) tests ;;
    quick) quick ;;
    bench:*) bench ${recipe#bench:} ;;
    evidence) bench c3 && bench driver && bench c2 && bench c5 ;;
    profile:*) profile ${recipe#profile:} ;;
    trace:driver) trace_driver ;;
    render_pmc) render_pmc ;;
    fsm) fsm ;;
    dataset:*) dataset ${recipe#dataset:} ;;
    ab) bash tools/ab.sh ;;
    occupancy) occupancy ;;
    *) echo "unknown recipe $recipe"; false ;;
  esac || exit $?
done
