set -o pipefail
# per-stage render clock (rclk) and triangle statistics (rstat) at C5 shape
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MMX_LIB_PATH=build/libmmx_rclk.so timeout -k 10 300 python -u tools/render_clock.py > gpurun_out/rclk.log 2>&1 || exit 1
cp gpurun_out/render_clock.json gpurun_out/render_clock_time.json
MMX_LIB_PATH=build/libmmx_rstat.so timeout -k 10 300 python -u tools/render_clock.py > gpurun_out/rstat.log 2>&1 || exit 1
cp gpurun_out/render_clock.json gpurun_out/render_clock_stats.json
cat gpurun_out/render_clock_time.json gpurun_out/render_clock_stats.json
