# Partitioned mode: GPU parity tests for it, then bench.py --partition (c5, 16,384 envs, 1 rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-part}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "partition" > $OUT/pytest_part.log 2>&1; rc=$?; echo "pytest part rc=$rc"; tail -2 $OUT/pytest_part.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --partition --steps ${STEPS:-3} --warmup 1 --decisions ${DEC:-16} > $OUT/bench_part.json 2> $OUT/bench_part.err; rc=$?; echo "bench part rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_part.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step']))"
