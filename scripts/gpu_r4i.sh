# round 4 (i): the bench kernel's wave-time split (one rocprofv3 --pmc pass per counter group, scripts/gpu_waitsplit.sh)
# and the SFL_PROFILE phase cycles of c2 at its stated 4,096 envs (configs[1])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r4h bash scripts/gpu_waitsplit.sh || exit 1
TAG=r4i_c2_4096_phase NOPMC=1 BENCH_ARGS="--config c2 --envs 4096 --verify-envs 0 --experimental" bash scripts/gpu_phase.sh || exit 1
TAG=r4i_c5pmc bash scripts/gpu_c5pmc.sh
