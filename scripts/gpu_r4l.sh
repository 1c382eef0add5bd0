# round 4 (l): the partitioned local step writes back only the changed train fields: partition GPU tests, the
# 8-rank rehearsal (throughput, parity) and its PMC write requests per env and round
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r4l STEPS="tests" PYTEST_ARGS="-k partition" bash scripts/gpu_r4.sh || exit 1
TAG=r4l STEPS="part" bash scripts/gpu_r4.sh || exit 1
TAG=r4l_c5pmc bash scripts/gpu_c5pmc.sh
