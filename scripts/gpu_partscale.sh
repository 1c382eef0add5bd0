# Partitioned-mode microbenchmarks (scripts/debug/part_micro) and the round cost vs env count.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-partscale}
mkdir -p $OUT
timeout -k 10 120 ./scripts/debug/part_micro > $OUT/micro.txt 2>&1; rc=$?; cat $OUT/micro.txt; [ $rc -eq 0 ] || exit $rc
for E in ${ENVS:-4096 8192 16384}; do
  timeout -k 10 300 python bench.py --partition --envs $E --steps 3 --warmup 1 --decisions 16 > $OUT/bench_$E.json 2> $OUT/bench_$E.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/bench_$E.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_$E.json'));print('E=$E  %.1fM/s  %.1f us/round' % (d['value']/1e6, d['ms_per_step']*1e3/d['config']['rounds_per_step']))"
done
