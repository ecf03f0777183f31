set -o pipefail
# one GPU call: interleaved A/B of the product library against $LIBS (tools/ab.sh, PMC=1 adds one SQ
# counter pass per library), the GPU suite (SUITE=1, no -x: every failure listed; a failing test is
# re-run with the first A/B library), tests $ALT_K (pytest -k) with each of $LIBS, and the f2
# host-path profile (DS=1, tools/gpu_ds_profile.sh); RTIME=1: render-only time per library
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
md5sum mujoco_manip_amd/libmmx.so $LIBS
if [ -n "$LIBS" ]; then TESTS=0 ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-512} bash tools/ab.sh || exit 1; fi
rc=0
if [ -n "$ALT_K" ]; then
  for lib in mujoco_manip_amd/libmmx.so $LIBS; do
    MMX_LIB_PATH=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -k "$ALT_K" -q --timeout 300 \
      --timeout-method thread > gpurun_out/alt_$(basename $lib .so).log 2>&1
    r=$?; echo "$lib [$ALT_K]: $(tail -1 gpurun_out/alt_$(basename $lib .so).log)"; [ $r -gt 1 ] && exit $r
  done
fi
if [ "${RTIME:-0}" = 1 ]; then  # render-only time (tools/render_time.py) per library
  for lib in mujoco_manip_amd/libmmx.so $LIBS; do
    MMX_LIB_PATH=$lib timeout -k 10 300 python -u tools/render_time.py > gpurun_out/rtime_$(basename $lib .so).log 2>&1 || exit 1
    echo "$lib render: $(grep -h '^{' gpurun_out/rtime_$(basename $lib .so).log | cut -c1-220)"
  done
fi
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -8 gpurun_out/gpu_tests.log
  [ $rc -gt 1 ] && exit $rc
  if [ $rc -eq 1 ] && [ -n "$LIBS" ]; then
    F=$(grep -h "^FAILED" gpurun_out/gpu_tests.log | sed 's/^FAILED \([^ ]*\).*/\1/' | tr '\n' ' ')
    MMX_LIB_PATH=${LIBS%% *} timeout -k 10 600 python -u -m pytest $F -q --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_tests_alt.log 2>&1; echo "with ${LIBS%% *}: $(tail -1 gpurun_out/gpu_tests_alt.log)"
  fi
fi
if [ "${DS:-1}" = 1 ]; then bash tools/gpu_ds_profile.sh || exit 1; fi
exit $rc
