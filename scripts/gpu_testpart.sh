# GPU parity suite, then the partitioned bench (c5, 16,384 envs, 1 rank) and the default bench without CPU legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-testpart}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K} > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --partition --steps 3 --warmup 1 --decisions 16 > $OUT/bench_part.json 2> $OUT/bench_part.err; rc=$?; echo "bench part rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_part.json'));print('  partition %.1fM/s  %.1f us/round, %s rounds/step' % (d['value']/1e6, d['ms_per_step']*1e3/d['config']['rounds_per_step'], d['config']['rounds_per_step']))"
timeout -k 10 600 python bench.py --partition --remote-rows --steps 3 --warmup 1 --decisions 16 > $OUT/bench_part_remote.json 2> $OUT/bench_part_remote.err; rc=$?; echo "bench part remote rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench_part_remote.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_part_remote.json'));print('  partition (all rows as messages) %.1fM/s  %.1f us/round' % (d['value']/1e6, d['ms_per_step']*1e3/d['config']['rounds_per_step']))"
timeout -k 10 600 python bench.py --partition --virtual-ranks 8 --steps 3 --warmup 1 --decisions 16 > $OUT/bench_part_v8.json 2> $OUT/bench_part_v8.err; rc=$?; echo "bench part v8 rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench_part_v8.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_part_v8.json'));print('  partition (8-rank traffic rehearsed) %.1fM/s  %.1f us/round, %s rounds/step' % (d['value']/1e6, d['ms_per_step']*1e3/d['config']['rounds_per_step'], d['config']['rounds_per_step']))"
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('  c3 %.1fM/s kernel %.3f ms' % (d['value']/1e6, d['roofline']['avg_kernel_ms']))"
