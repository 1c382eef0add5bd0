# round 5: c3 (65,536 envs) by lane-group size (SFL_WAVE_G) on the product build and on a whole-library build with
# the register-minimising scheduler
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p $OUT
for LG in ${RUNS:-libsfl:16 libsfl:32 libsfl_minreg:32 libsfl_minreg:64 libsfl:16}; do
  L=${LG%%:*}; GS=${LG#*:}
  SFL_WAVE_G=$GS SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --experimental --verify-envs 4 --sustain-seconds 0 > $OUT/${L}_g$GS.json 2> $OUT/${L}_g$GS.err; rc=$?
  [ $rc -eq 0 ] || { echo "$L G=$GS rc=$rc"; tail -3 $OUT/${L}_g$GS.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/${L}_g$GS.json'));print('$L G=$GS  %.1fM/s kernel %.3f ms parity %s %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity'), d['roofline']['kernel']))"
done
