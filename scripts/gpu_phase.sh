# Phase-cycle profile (SFL_PROFILE build: reset/tick/decide/post wall cycles per wave) + PMC instruction mix.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-phase}
mkdir -p $OUT
SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_profile.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/phase_bench.json 2> $OUT/phase_bench.err; rc=$?; echo "phase rc=$rc"; grep "sfl" $OUT/phase_bench.err
[ $rc -eq 0 ] || exit $rc
[ -n "$NOPMC" ] && exit 0
TAG=${TAG:-phase}/mix bash scripts/gpu_pmc.sh
