# round 5: cohorts at the partitioned leg's size (2,048 envs per GPU, 256 decisions per step) and at 4,096 / 8,192
# envs, on the one-GPU 8-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ac}
mkdir -p $OUT
for EC in ${RUNS:-2048:1 2048:2 2048:3 4096:1 4096:2 4096:3 8192:1 8192:3 2048:1}; do
  E=${EC%%:*}; C=${EC#*:}
  timeout -k 10 300 python bench.py --partition --steps 4 --warmup 2 --decisions 256 --virtual-ranks 8 --envs $E --cohorts $C --verify-envs 4 > $OUT/p_${E}_$C.json 2> $OUT/p_${E}_$C.err; rc=$?
  [ $rc -eq 0 ] || { echo "envs $E cohorts $C rc=$rc"; tail -3 $OUT/p_${E}_$C.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/p_${E}_$C.json'));r=d['config']['rounds_per_step'];print('envs $E cohorts $C  %.1fM/s  %.2f ms/step  %.1f us/round  parity %s' % (d['value']/1e6, d['ms_per_step'], 1e3*d['ms_per_step']/r, d.get('parity')))"
done
