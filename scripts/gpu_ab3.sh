# A/B/C of alternative builds (SFL_LIB) on one box for three workloads: the c3 bench, c5 fused
# (8,192 envs, 256 decisions per env per step) and the c5 partitioned mode (16,384 envs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab3}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  export SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu > $OUT/${L}_c3.json 2> $OUT/${L}_c3.err || exit 1
  timeout -k 10 300 python bench.py --config c5 --envs 8192 --decisions 256 --steps 3 --warmup 1 --no-cpu > $OUT/${L}_c5.json 2> $OUT/${L}_c5.err || exit 1
  timeout -k 10 300 python bench.py --partition --steps 3 --warmup 1 --decisions 16 > $OUT/${L}_part.json 2> $OUT/${L}_part.err || exit 1
  python -c "
import json
r=[json.load(open('$OUT/${L}_%s.json' % w))['value']/1e6 for w in ('c3','c5','part')]
print('$L c3 %.1fM c5 %.1fM part %.2fM' % tuple(r))"
done
