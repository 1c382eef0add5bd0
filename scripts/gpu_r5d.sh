# round 5, call D: the partitioned round with the block-cooperative owner kernel -- partition GPU tests, the
# 8-rank rehearsal and its kernel stats -- then call C's duplicate-write A/B and phase laps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "partition" > $OUT/pytest_part.log 2>&1; rc=$?
echo "pytest part rc=$rc"; tail -2 $OUT/pytest_part.log; [ $rc -eq 0 ] || exit $rc
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
timeout -k 10 300 python bench.py $P --verify-envs 4 > $OUT/part.json 2> $OUT/part.err; rc=$?; echo "part rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/part.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/part.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/part_prof -o ktrace --output-format csv -- python bench.py $P --verify-envs 0 > $OUT/part_prof.json 2>/dev/null; rc=$?; echo "part ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
head -5 $OUT/part_prof/ktrace_kernel_stats.csv | cut -c1-180
TAG=${TAG:-r5d} bash scripts/gpu_r5c.sh
