# round 5, call I: mf_propose without the f64 conversion and the 64-bit `%` (A/B against SFL_MF_FASTMOD=0 on the
# same box, c3 and c2 at 4,096 envs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r5i STEPS="ab" LIBS="libsfl libsfl_mfold libsfl libsfl_mfold" BSTEPS=6 VERIFY_ENVS=8 bash scripts/gpu_r4.sh || exit 1
TAG=r5i_c2 STEPS="ab" LIBS="libsfl libsfl_mfold libsfl libsfl_mfold" BSTEPS=10 VERIFY_ENVS=8 BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh || exit 1
