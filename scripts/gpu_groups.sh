# A/B of the lane-group size (SFL_WAVE_G = 64 / 32 / 16): GPU parity tests under each grouped size,
# then the c3 bench for each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-groups}
mkdir -p $OUT
for g in ${TEST_G:-16 32}; do
  SFL_WAVE_G=$g timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K} > $OUT/pytest_g$g.log 2>&1; rc=$?; echo "pytest G=$g rc=$rc"; tail -2 $OUT/pytest_g$g.log
  [ $rc -eq 0 ] || exit $rc
done
for g in ${BENCH_G:-64 32 16}; do
  SFL_WAVE_G=$g timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/bench_g$g.json 2> $OUT/bench_g$g.err; rc=$?; echo "bench G=$g rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/bench_g$g.json'));print('  %.1fM/s kernel %.3f ms %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d['roofline']['kernel']))"
done
