# round 5, call F: tick-hold rules for the two-envs-per-wavefront shape (c2 at its 4,096 envs, G = 32): the
# product rule never holds a ticking group at G = 32 (it needs two other groups deciding); HOLD=1 ticks a
# waiting group only when the other group is not deciding (or, REMMIN, has enough decisions left).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r5f} STEPS="ab" LIBS="${LIBS:-libsfl libsfl_hold1 libsfl_hold1r0 libsfl_hold1r2 libsfl}" BSTEPS=10 VERIFY_ENVS=8 BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh
