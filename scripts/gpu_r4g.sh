# round 4 (g): round-end evidence for the product build -- smoke, default bench, rocprofv3 kernel stats, the
# HBM-traffic PMC passes and the wave-time split (scripts/gpu_final.sh), then the SFL_PROFILE phase cycles of
# c2 at its stated 4,096 envs (configs[1])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r4g_final bash scripts/gpu_final.sh || exit 1
TAG=r4g_c2_4096_phase NOPMC=1 BENCH_ARGS="--config c2 --envs 4096 --verify-envs 0 --experimental" bash scripts/gpu_phase.sh
