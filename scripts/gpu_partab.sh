# A/B of library builds on the partitioned bench (c5, 16,384 envs, 1 rank): LIBS="libsfl libsfl_x ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-partab}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --partition --steps ${STEPS:-3} --warmup 1 --decisions 16 > $OUT/$L.json 2> $OUT/$L.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/$L.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/$L.json'));print('$L  %.1fM/s  %.1f us/round' % (d['value']/1e6, d['ms_per_step']*1e3/d['config']['rounds_per_step']))"
done
