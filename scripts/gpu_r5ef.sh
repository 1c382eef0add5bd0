# round 5: calls E and F in one box: partition laps, the c2 tick-hold A/B, then the GPU learning curve
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5e
mkdir -p $OUT
SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_profile.so timeout -k 10 300 python bench.py --partition --steps 1 --warmup 1 --decisions 256 --virtual-ranks 8 --verify-envs 0 --experimental > $OUT/part_prof.json 2> $OUT/part_prof.err; rc=$?
echo "part prof rc=$rc"; grep "sfl" $OUT/part_prof.err | tail -4; [ $rc -eq 0 ] || exit $rc
TAG=r5f bash scripts/gpu_r5f.sh || exit 1
timeout -k 10 1000 python -u scripts/learning_curve.py $OUT/lc_gpu.json --compare profiles/r05_learning_curve_sweep_host.json.gz > $OUT/lc_gpu.log 2>&1; rc=$?
echo "learning curve rc=$rc"; tail -3 $OUT/lc_gpu.log; [ $rc -eq 0 ] || exit $rc
