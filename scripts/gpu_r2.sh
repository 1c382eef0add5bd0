# Round-2 GPU pass: parity tests (incl. the bench-horizon and API tests), smoke, default bench,
# then optional phase profile (SFL_PROFILE build) and store-drop A/B builds (timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 1000 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K} > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
for L in ${LIBS}; do
  SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/$L.json 2> $OUT/$L.err; rc=$?; echo "$L rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/$L.json'));print('  %.1fM/s kernel %.3f ms' % (d['value']/1e6, d['roofline']['avg_kernel_ms']))"
  grep "sfl" $OUT/$L.err | tail -2
done
