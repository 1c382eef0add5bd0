# round 5, call G: the partitioned local step with the observe pass's prefetch record carried to the apply pass
# (and no owned-table offsets for other ranks' rows): partition GPU tests, then the 8-rank rehearsal A/B against the
# previous build (libsfl_r5d.so) on the same box, and the kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "partition" > $OUT/pytest_part.log 2>&1; rc=$?
echo "pytest part rc=$rc"; tail -2 $OUT/pytest_part.log; [ $rc -eq 0 ] || exit $rc
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
for L in libsfl; do
  SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py $P --verify-envs 4 --experimental > $OUT/part_$L.json 2> $OUT/part_$L.err; rc=$?; echo "part $L rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/part_$L.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/part_$L.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/part_prof -o ktrace --output-format csv -- python bench.py $P --verify-envs 0 > $OUT/part_prof.json 2>/dev/null; rc=$?; echo "part ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
head -5 $OUT/part_prof/ktrace_kernel_stats.csv | cut -c1-180
