set -o pipefail
# f2 host-path split: collect-only (--no-write) and collect + write, each with a cProfile of the
# collecting thread; logs / profiles under gpurun_out/ds/
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/ds; mkdir -p $OUT
E=${ENVS:-4096}; S=${SIZE:-128}
timeout -k 10 300 python -u tools/dataset_bench.py --num-envs $E --episodes $E --image-size $S --no-write \
  --cprofile $OUT/prof_nowrite_${E}_${S}.txt --out $OUT/nowrite_${E}_${S}.json > $OUT/nowrite.log 2>&1 && \
timeout -k 10 300 python -u tools/dataset_bench.py --num-envs $E --episodes $E --image-size $S \
  --cprofile $OUT/prof_write_${E}_${S}.txt --out $OUT/write_${E}_${S}.json > $OUT/write.log 2>&1
rc=$?; grep -h frames_per_s $OUT/*.json; exit $rc
