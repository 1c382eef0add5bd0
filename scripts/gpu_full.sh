# GPU round: parity tests, smoke, entry-point scripts, bench, rocprof kernel stats + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python test_model.py $OUT/test_model --episodes 5 > $OUT/test_model.log 2>&1; echo "test_model rc=$?"; tail -4 $OUT/test_model.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
[ -n "$NOPROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_bench.json 2>/dev/null; rc=$?; echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$N -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1; rc=$?; echo "pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
