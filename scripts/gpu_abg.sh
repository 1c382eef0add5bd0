# A/B: bench.py (c3 default workload, no CPU legs) for each library in LIBS x lane-group size in GS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abg}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  for g in ${GS:-64}; do
    SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so SFL_WAVE_G=$g timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/${L}_g$g.json 2> $OUT/${L}_g$g.err; rc=$?
    [ $rc -eq 0 ] || { echo "$L G=$g rc=$rc"; tail -5 $OUT/${L}_g$g.err; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/${L}_g$g.json'));print('$L G=$g: %.1fM/s kernel %.3f ms %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d['roofline']['kernel']))"
  done
done
