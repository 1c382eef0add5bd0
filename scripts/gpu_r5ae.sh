# round 5: the driver's N > 1 path rehearsed again on one GPU over gloo (RCCL refuses two ranks on one device) with
# the final build: bench.py --gpus 2 / 4 -- env-sharded step, parity, the sustained window, the partitioned leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ae}
mkdir -p $OUT
for N in 2 4; do
  SFL_DIST_BACKEND=gloo SFL_DEVICE=0 timeout -k 10 600 python bench.py --gpus $N --envs 8192 --steps 3 --warmup 1 --sustain-seconds 3 > $OUT/gpus$N.json 2> $OUT/gpus$N.err; rc=$?
  echo "gpus $N rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/gpus$N.err; exit $rc; }
  python -c "
import json; d=[json.loads(l) for l in open('$OUT/gpus$N.json') if l.startswith('{')][0]; p=d['partition_leg']; s=d['sustained']
print('  env-sharded %.1f M/s world %d parity %s sustained %.1f M/s over %d steps | leg %s' % (d['value']/1e6, d['world_size'], d['parity'], s['value']/1e6, s['steps'], {k: p.get(k) for k in ('value','world_size','backend','rounds_per_step','cohorts','collectives_per_round','deferrals','parity','parity_envs_checked','error')}))"
done
