set -o pipefail
# launch-shape experiment: driver-config windows (--steps 20 --warmup 5, 5 repeats) and 512-step
# windows for several MMX_FUSE values; plus a kernel trace of the driver config (dispatch timeline)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fuse; : > gpurun_out/fuse/res.txt
for f in 16 10 20 32; do
  MMX_FUSE=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/fuse/d$f.log 2>&1 || { tail gpurun_out/fuse/d$f.log; exit 1; }
  echo "driver fuse=$f $(grep -h '^{' gpurun_out/fuse/d$f.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), [round(v) for v in d["repeats"]["values"]], round(d["roofline"]["kernel_ms"],2), round(d["roofline"]["span_ms_per_launch_round"],2))')" >> gpurun_out/fuse/res.txt
done
for f in 16 32; do
  MMX_FUSE=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 512 --warmup 64 --repeats 2 > gpurun_out/fuse/b$f.log 2>&1 || exit 1
  echo "512 fuse=$f $(grep -h '^{' gpurun_out/fuse/b$f.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), [round(v) for v in d["repeats"]["values"]], round(d["roofline"]["kernel_ms"],2), round(d["roofline"]["span_ms_per_launch_round"],2))')" >> gpurun_out/fuse/res.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/fuse/kt.log 2>&1 || exit 1
f=$(find /tmp/kt -name "*kernel_trace.csv" | head -1); python3 - "$f" > $GRAFT_REPO_ROOT/gpurun_out/fuse/timeline.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'env_step' in r['Kernel_Name']]
t0 = min(int(r['Start_Timestamp']) for r in rows)
print(list(rows[0].keys()))
for r in rows: print(r.get('Queue_Id', r.get('Stream_Id','?')), r.get('Stream_Id','?'), (int(r['Start_Timestamp'])-t0)/1e6, (int(r['End_Timestamp'])-t0)/1e6, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6)
PY
cat $GRAFT_REPO_ROOT/gpurun_out/fuse/res.txt
