# round 5, call K: block sizes of the partitioned round's compaction (SFL_COMPACT_BLOCK) and owner
# (SFL_OWN_CHUNK) kernels: the 8-rank rehearsal A/B on one box, each with its parity check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5k}
mkdir -p $OUT
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
for L in ${LIBS:-libsfl libsfl_cb512 libsfl_cb1024 libsfl_oc128 libsfl_oc512 libsfl}; do
  SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so timeout -k 10 300 python bench.py $P --verify-envs 4 --experimental > $OUT/part_$L.json 2> $OUT/part_$L.err; rc=$?; echo "part $L rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/part_$L.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/part_$L.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
done
