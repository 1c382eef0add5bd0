# round 5: c2 at its 4,096 envs by lane-group size (SFL_WAVE_G: 16 / 32 / 64 lanes per env) on the product build
# and on a whole-library register-minimising-scheduler build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5aa}
mkdir -p $OUT
for L in libsfl libsfl_minreg; do
  for GS in 32 64 16 32; do
    SFL_WAVE_G=$GS SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py --config c2 --envs 4096 --steps 10 --warmup 2 --no-cpu --experimental --verify-envs 4 --sustain-seconds 0 > $OUT/${L}_g$GS.json 2> $OUT/${L}_g$GS.err; rc=$?
    [ $rc -eq 0 ] || { echo "$L G=$GS rc=$rc"; tail -3 $OUT/${L}_g$GS.err; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/${L}_g$GS.json'));print('$L G=$GS  %.1fM/s kernel %.3f ms parity %s %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity'), d['roofline']['kernel']))"
  done
done
