# round 5, call L: the 8-rank partition rehearsal's round time against the env count (generations of resident
# waves: 12 envs per CU x 256 CUs = 3,072 per generation; the owned Q rows grow with the envs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5l}
mkdir -p $OUT
for E in ${ENVS:-3072 6144 12288 15360 16384}; do
  timeout -k 10 300 python bench.py --partition --steps 2 --warmup 1 --decisions 512 --virtual-ranks 8 --envs $E --verify-envs 0 > $OUT/part_$E.json 2> $OUT/part_$E.err; rc=$?; echo "envs $E rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/part_$E.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/part_$E.json'));r=d['config']['rounds_per_step'];print('  %.1fM/s  %.1f ms/step  rounds/step %s  us/round %.1f  us/round/gen %.1f' % (d['value']/1e6, d['ms_per_step'], r, 1e3*d['ms_per_step']/r, 1e3*d['ms_per_step']/r/(-(-$E//3072))))"
done
