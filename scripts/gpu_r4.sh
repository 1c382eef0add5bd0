# Round 4 check: GPU suite, product bench, SFL_PROFILE phase laps (libsfl_profile.so), each step timed.
# Usage: TAG=name STEPS="tests bench prof" bash scripts/gpu_r4.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4}
mkdir -p $OUT
for S in ${STEPS:-tests bench prof}; do
  case $S in
    tests)
      timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 300 python bench.py --steps ${BSTEPS:-10} --warmup 2 --no-cpu ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
      python -c "import json;d=json.load(open('$OUT/bench.json'));print('  %.1fM/s kernel %.3f ms parity %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity')))" ;;
    prof)
      SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_profile.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --verify-envs 0 --experimental ${BENCH_ARGS} > $OUT/prof.json 2> $OUT/prof.err; rc=$?
      echo "prof rc=$rc"; grep "sfl" $OUT/prof.err | tail -4; [ $rc -eq 0 ] || exit $rc ;;
    part)
      timeout -k 10 300 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --verify-envs 4 --virtual-ranks 8 ${BENCH_ARGS} > $OUT/part.json 2> $OUT/part.err; rc=$?
      echo "part rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/part.err; exit $rc; }
      python -c "import json;d=json.load(open('$OUT/part.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))" ;;
    ab)
      for L in ${LIBS}; do
        SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --steps ${BSTEPS:-10} --warmup 2 --no-cpu --experimental --verify-envs ${VERIFY_ENVS:-4} ${BENCH_ARGS} > $OUT/ab_$L.json 2> $OUT/ab_$L.err; rc=$?
        echo "ab $L rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/ab_$L.err; exit $rc; }
        python -c "import json;d=json.load(open('$OUT/ab_$L.json'));print('  %.1fM/s kernel %.3f ms parity %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity')))"
      done ;;
  esac
done
