# C5 (graph-partitioned) round study: partition GPU tests, the 8-rank rehearsal and the message path at
# 1,024 decisions, a kernel trace of the rehearsal, and the SFL_PROFILE build's local-step phase cycles.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c5}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "partition" > $OUT/pytest_part.log 2>&1; rc=$?; echo "pytest part rc=$rc"; tail -2 $OUT/pytest_part.log
[ $rc -eq 0 ] || exit $rc
fi
for M in "virtual8:--virtual-ranks 8" "remote:--remote-rows"; do
  N=${M%%:*}; A=${M#*:}
  timeout -k 10 300 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --verify-envs 4 $A ${BENCH_ARGS} > $OUT/bench_$N.json 2> $OUT/bench_$N.err; rc=$?; echo "bench $N rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/bench_$N.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_$N.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --partition --steps 2 --warmup 1 --decisions 128 --verify-envs 0 --virtual-ranks 8 ${BENCH_ARGS} > $OUT/ktrace_bench.json 2> $OUT/ktrace_bench.err; rc=$?; echo "ktrace rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/ktrace_bench.err; exit $rc; }
if [ -f network-distributed-q-learning_amd/libsfl_profile.so ]; then
SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_profile.so timeout -k 10 300 python bench.py --partition --steps 1 --warmup 0 --decisions 16 --verify-envs 0 --experimental --virtual-ranks 8 ${BENCH_ARGS} > $OUT/phase.json 2> $OUT/phase.err; rc=$?; echo "phase rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/phase.err; exit $rc; }
grep "sfl" $OUT/phase.err | tail -6
fi
