set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dsk
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dsk/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 --no-write --out $GRAFT_REPO_ROOT/gpurun_out/dsk/nowrite.json > $GRAFT_REPO_ROOT/gpurun_out/dsk/log.txt 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; find gpurun_out/dsk -name "*stats*" | head; for f in $(find gpurun_out/dsk -name "*kernel_stats.csv"); do head -12 $f | cut -c1-200; done; for f in $(find gpurun_out/dsk -name "*memory_copy_stats.csv"); do head -8 $f | cut -c1-200; done; grep frames_per_s gpurun_out/dsk/nowrite.json; exit $rc
