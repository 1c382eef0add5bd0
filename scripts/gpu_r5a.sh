# round 5, call A: (1) FETCH_SIZE / WRITE_SIZE calibration on the bench kernel's access shapes
# (scripts/calib/fetch_calib.bin, one --pmc pass per counter), (2) configs[1] (c2, 4,096 envs) bench line
# + kernel stats + HBM-traffic PMC + wave-time split, (3) the list of available counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5a}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1; echo "list rc=$?"
timeout -k 10 120 scripts/calib/fetch_calib.bin > $OUT/calib.json; rc=$?; echo "calib rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" ${CALIB_EXTRA}; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $OUT/calib_$N -o pmc --output-format csv -- scripts/calib/fetch_calib.bin > /dev/null 2>$OUT/calib_$N.err; rc=$?
  echo "calib pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/calib/fetch_calib.py $OUT $OUT/fetch_calib.json || exit 1
# configs[1]: c2 at its stated 4,096 envs
B="--config c2 --envs 4096"
timeout -k 10 300 python bench.py $B --steps 10 --warmup 2 --no-cpu > $OUT/c2_bench.json 2> $OUT/c2_bench.err; rc=$?; echo "c2 bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/c2_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_prof -o ktrace --output-format csv -- python bench.py $B --steps 10 --warmup 2 --no-cpu --verify-envs 0 > $OUT/c2_prof_bench.json 2>/dev/null; rc=$?; echo "c2 ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/c2/pmc_$N -o pmc --output-format csv -- python bench.py $B --steps 3 --warmup 1 --no-cpu --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "c2 pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG:-r5a}/c2 BENCH_ARGS="$B --verify-envs 0" DEC=$((4096*1024)) bash scripts/gpu_waitsplit.sh || exit 1
