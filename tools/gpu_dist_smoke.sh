set -o pipefail
# smoke() + a 2-rank rehearsal of the N>1 bench path on one GPU (gloo, ranks share device 0)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --steps 50 --warmup 10 --dist-backend gloo --share-device --envs-per-gpu 2048 > gpurun_out/dist2.log 2>&1; rc=$?
grep -h "^{" gpurun_out/dist2.log | cut -c 1-300; exit $rc
