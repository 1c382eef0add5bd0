# round 5, final evidence for the committed build: parts 1 and 2 in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r5y} bash scripts/gpu_r5z1.sh || exit 1
TAG=${TAG:-r5y} bash scripts/gpu_r5z2.sh || exit 1
