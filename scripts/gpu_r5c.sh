# round 5, call C: the post step's writes priced by duplicate-write builds (results unchanged; the bound on
# what the round-4 verdict's slot write-back cache can gain), phase laps of c3 and of c2 at its 4,096 envs
# (libsfl_profile.so), and the sweep learning curve through libsfl.so compared with the host build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5c}
mkdir -p $OUT
TAG=${TAG:-r5c} STEPS="ab" LIBS="${LIBS:-libsfl libsfl_ab_slot2 libsfl_ab_qst2 libsfl_ab_touch2 libsfl}" BSTEPS=6 VERIFY_ENVS=4 bash scripts/gpu_r4.sh || exit 1
TAG=${TAG:-r5c}/prof_c3 STEPS="prof" bash scripts/gpu_r4.sh || exit 1
TAG=${TAG:-r5c}/prof_c2 STEPS="prof" BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh || exit 1
if [ -n "$LC" ]; then
  timeout -k 10 900 python -u scripts/learning_curve.py $OUT/lc_gpu.json --compare profiles/r05_learning_curve_sweep_host.json.gz > $OUT/lc_gpu.log 2>&1; rc=$?
  echo "learning curve rc=$rc"; tail -3 $OUT/lc_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
