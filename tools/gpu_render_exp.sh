set -o pipefail
# render experiment: the render GPU tests on the working tree, then the render-only A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_render.py tests/test_png.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/render_tests.log 2>&1; rc=$?
tail -3 gpurun_out/render_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/render_ab3.sh
