# Partitioned-mode breakdown: kernel trace of bench.py --partition (per-kernel time per round), then
# the SFL_PROFILE build's phase cycles of the local step (libsfl_profile.so, scripts/build_variants.sh PROFILE).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-partprof}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --partition --steps 3 --warmup 1 --decisions 16 ${BENCH_ARGS} > $OUT/bench_part.json 2> $OUT/bench_part.err; rc=$?; echo "ktrace rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit $rc; }
cat $OUT/bench_part.json
if [ -f network-distributed-q-learning_amd/libsfl_profile.so ]; then
SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_profile.so timeout -k 10 300 python bench.py --partition --steps 1 --warmup 0 --decisions 16 ${BENCH_ARGS} > $OUT/phase.json 2> $OUT/phase.err; rc=$?; echo "phase rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/phase.err; exit $rc; }
grep "sfl" $OUT/phase.err | tail -4
fi
