# round 4 (k): the launcher's real spawn path on the GPU box -- bench.py --gpus 2 with both ranks on GPU 0 over
# gloo (SFL_DIST_BACKEND=gloo SFL_DEVICE=0: a rehearsal of the driver's N-GPU run, not the RCCL transport) --
# and the default bench with the larger parity sample (32 envs per rank); the --gpus 2 line carries the
# partitioned leg (configs[4] over the same process group)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4k; mkdir -p $OUT
SFL_DIST_BACKEND=gloo SFL_DEVICE=0 timeout -k 10 600 python bench.py --gpus 2 --envs 16384 --steps 20 --warmup 2 --no-cpu > $OUT/gpus2.json 2> $OUT/gpus2.err; rc=$?; echo "gpus2 rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/gpus2.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/gpus2.json'));print('  %.1fM/s n_gpus %s world %s backend %s devices %s parity %s checked %s' % (d['value']/1e6, d['n_gpus'], d['world_size'], d['backend'], d['devices'], d.get('parity'), d.get('parity_envs_checked'))); print('  leg', d.get('partition_leg'))"
T0=$(date +%s); timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('  %.1fM/s parity %s checked %s oracle %s' % (d['value']/1e6, d.get('parity'), d.get('parity_envs_checked'), d['cpu_oracle_baseline'].get('oracle_parity',{}).get('result')))"
echo "  bench wall $(( $(date +%s) - T0 )) s"
