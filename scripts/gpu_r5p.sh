# round 5, call P: LLVM AMDGPU scheduler strategies (whole-library -mllvm -amdgpu-sched-strategy=...) on every
# bench workload: (C3=1: c3,) c2 at 4,096 and 65,536 envs, c5 fused at 16,384 envs, and the 8-rank partition rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5p}
mkdir -p $OUT
L3="${LIBS:-libsfl libsfl_minreg libsfl_mmc libsfl}"
[ -n "$C3" ] && { TAG=${TAG:-r5p}/c3 STEPS=ab LIBS="$L3" BSTEPS=6 bash scripts/gpu_r4.sh || exit 1; }
TAG=${TAG:-r5p}/c2_4096 STEPS=ab LIBS="$L3" BSTEPS=10 BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh || exit 1
TAG=${TAG:-r5p}/c2_65536 STEPS=ab LIBS="$L3" BSTEPS=6 BENCH_ARGS="--config c2 --envs 65536" bash scripts/gpu_r4.sh || exit 1
TAG=${TAG:-r5p}/c5_16384 STEPS=ab LIBS="$L3" BSTEPS=4 BENCH_ARGS="--config c5 --envs 16384" bash scripts/gpu_r4.sh || exit 1
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
for L in $L3; do
  SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py $P --verify-envs 4 --experimental > $OUT/part_$L.json 2> $OUT/part_$L.err; rc=$?; echo "part $L rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/part_$L.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/part_$L.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
done
