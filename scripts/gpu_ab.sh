# A/B of alternative builds (SFL_LIB, accepted with --experimental) on one box: bench (+ optional SQ PMC pass)
# for each; the product library first, with its post-run parity check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  export SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so
  V="--verify-envs ${VERIFY_ENVS:-0} --experimental"; [ "$L" = "libsfl" ] && V=""
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu $V ${BENCH_ARGS} > $OUT/${L}.json 2> $OUT/${L}.err; rc=$?; echo "$L bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/${L}.json'));print('  %.1fM/s kernel %.3f ms parity %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity')))"
  if [ -n "$PMC" ]; then
    timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $OUT/pmc_$L -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --verify-envs 0 --experimental ${BENCH_ARGS} > /dev/null 2>&1; rc=$?; echo "  pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python scripts/pmc_per_dec.py $OUT/pmc_$L | sed 's/^/  /'
  fi
done
