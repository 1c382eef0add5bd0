# Round-end measurement of the product build (tests run separately): smoke, default bench, rocprofv3 kernel
# stats, HBM traffic PMC passes and the wave-time split passes (bench roofline.traffic / roofline.issue).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --verify-envs 0 > $OUT/prof_bench.json 2>/dev/null; rc=$?; echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$N -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG:-final} bash scripts/gpu_waitsplit.sh
