# round 5, call J: the driver's N > 1 path rehearsed on one GPU over gloo (RCCL refuses two ranks on one device):
# bench.py --gpus 2 and --gpus 4 launch their ranks, time the env-sharded step, check parity, then run the
# partitioned leg (one message all-to-all + one reply all-to-all per round) with its parity check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5j}
mkdir -p $OUT
for N in 2 4; do
  SFL_DIST_BACKEND=gloo SFL_DEVICE=0 timeout -k 10 600 python bench.py --gpus $N --envs 8192 --steps 3 --warmup 1 > $OUT/gpus$N.json 2> $OUT/gpus$N.err; rc=$?
  echo "gpus $N rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/gpus$N.err; exit $rc; }
  python -c "
import json; d=[json.loads(l) for l in open('$OUT/gpus$N.json') if l.startswith('{')][0]; p=d['partition_leg']
print('  env-sharded %.1f M/s world %d parity %s | leg %s' % (d['value']/1e6, d['world_size'], d['parity'], {k: p.get(k) for k in ('value','world_size','backend','rounds_per_step','segment_records','collectives_per_round','deferrals','parity','parity_envs_checked','error')}))"
done
# c3: the tick rule's REMMIN re-measured on the current kernel (product 5)
TAG=${TAG:-r5j}_rem STEPS="ab" LIBS="libsfl libsfl_rem3 libsfl_rem4 libsfl_rem7 libsfl" BSTEPS=6 VERIFY_ENVS=4 bash scripts/gpu_r4.sh || exit 1
