# round 4 (j): occupancy A/Bs where the batch, not the registers, sets the waves per SIMD: the G = 32 shapes
# compiled for 2 waves per SIMD (no spills) on c2 at its stated 4,096 envs, and the partitioned local step
# (k_wave2_part) at 4 waves per SIMD (128 VGPRs, spilled) on the 8-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd
TAG=r4j_c2_4096 STEPS="ab" BENCH_ARGS="--config c2 --envs 4096" LIBS="libsfl libsfl_g32o2 libsfl libsfl_g32o2" bash scripts/gpu_r4.sh || exit 1
OUT=gpurun_out/r4j_part; mkdir -p $OUT
for V in libsfl libsfl_w2p4 libsfl libsfl_w2p4; do
  SFL_LIB=$L/$V.so timeout -k 10 300 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --verify-envs 2 --virtual-ranks 8 --experimental > $OUT/$V.json 2> $OUT/$V.err; rc=$?
  echo "part $V rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$V.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/$V.json'));print('  %.1fM/s parity %s' % (d['value']/1e6, d.get('parity')))"
done
