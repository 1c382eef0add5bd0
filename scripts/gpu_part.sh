# Graph-partitioned mode on one GPU: bench (configs[4] shape, one rank) after the parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-part}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k partitioned > $OUT/pytest_part.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_part.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --partition --steps 3 --warmup 1 --decisions ${DEC:-16} ${BENCH_ARGS} > $OUT/bench_part.json 2> $OUT/bench_part.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench_part.json; tail -3 $OUT/bench_part.err
[ -n "$PROF" ] || exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_part -o ktrace --output-format csv -- python bench.py --partition --steps 3 --warmup 1 --decisions ${DEC:-16} ${BENCH_ARGS} > $OUT/prof_bench_part.json 2>/dev/null; echo "ktrace rc=$?"
