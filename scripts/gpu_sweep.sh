# Tuning sweep: alternative builds (SFL_LIB) and env counts, bench only (no parity tests).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sweep
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  for E in ${ENVS:-65536}; do
    SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --envs $E > $OUT/${L}_$E.json 2> $OUT/${L}_$E.err
    rc=$?; echo "$L E=$E rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('$OUT/${L}_$E.json'));print('  %.1fM/s kernel %.2f ms' % (d['value']/1e6, d['roofline']['avg_kernel_ms']))"
  done
done
