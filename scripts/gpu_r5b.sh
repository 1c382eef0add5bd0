# round 5, call B: the GPU suite on the ABI-8 partitioned exchange (one message all-to-all, one owner kernel),
# the 8-rank partition rehearsal + its kernel stats, and the memory-side request-size counters
# (TCC_EA0_RDREQ_32B/64B/128B, ...) on the calibration kernels and on the c3 bench kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
timeout -k 10 300 python bench.py $P --verify-envs 4 > $OUT/part.json 2> $OUT/part.err; rc=$?; echo "part rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/part.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/part.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/part_prof -o ktrace --output-format csv -- python bench.py $P --verify-envs 0 > $OUT/part_prof.json 2>/dev/null; rc=$?; echo "part ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
head -8 $OUT/part_prof/ktrace_kernel_stats.csv | cut -c1-200
EA1="TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"
EA2="TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"
EA3="TCC_EA0_WRREQ_DRAM TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ_ATOMIC_DRAM TCC_EA0_WRREQ_ATOMIC_DRAM_32B"
timeout -k 10 120 scripts/calib/fetch_calib.bin > $OUT/calib.json; rc=$?; echo "calib rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for C in "$EA1" "$EA2" "$EA3" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $OUT/calib_$i -o pmc --output-format csv -- scripts/calib/fetch_calib.bin > /dev/null 2>$OUT/calib_$i.err; rc=$?
  echo "calib pmc $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/calib_$i.err; exit $rc; }
done
python scripts/calib/fetch_calib.py $OUT $OUT/fetch_calib.json || exit 1
i=0
for C in "$EA1" "$EA2" "$EA3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/c3ea/pmc_ea$i -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --verify-envs 0 > /dev/null 2>$OUT/c3ea_$i.err; rc=$?
  echo "c3 pmc ea$i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/c3ea_$i.err; exit $rc; }
done
python scripts/pmc_per_dec.py "$OUT/c3ea/pmc_*" > $OUT/c3ea/per_dec.txt; cat $OUT/c3ea/per_dec.txt
