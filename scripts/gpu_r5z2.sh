# round 5, final evidence (part 2): configs[1] (c2 at its 4,096 envs) with kernel stats, traffic PMC and the
# wave-time split; c2 at 65,536 envs; c5 fused at 16,384 envs; the 8-rank partition rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5z}
mkdir -p $OUT
B="--config c2 --envs 4096"
timeout -k 10 300 python bench.py $B --steps 10 --warmup 2 --no-cpu > $OUT/c2_bench.json 2> $OUT/c2_bench.err; rc=$?; echo "c2 bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/c2_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_prof -o ktrace --output-format csv -- python bench.py $B --steps 10 --warmup 2 --no-cpu --sustain-seconds 0 --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "c2 ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/c2/pmc_$N -o pmc --output-format csv -- python bench.py $B --steps 3 --warmup 1 --no-cpu --sustain-seconds 0 --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "c2 pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG:-r5z}/c2 BENCH_ARGS="$B --verify-envs 0" DEC=$((4096*1024)) bash scripts/gpu_waitsplit.sh || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu > $OUT/c2_65536_bench.json 2> $OUT/c2_65536.err; rc=$?; echo "c2 65536 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --envs 16384 --steps 4 --warmup 1 --no-cpu > $OUT/c5_fused_bench.json 2> $OUT/c5_fused.err; rc=$?; echo "c5 fused rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8 --verify-envs 4 > $OUT/part.json 2> $OUT/part.err; rc=$?; echo "part rc=$rc"; [ $rc -eq 0 ] || exit $rc
for f in c2_bench c2_65536_bench c5_fused_bench part; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('  $f %.1fM/s  %.2f ms/step parity %s' % (d['value']/1e6, d['ms_per_step'], d.get('parity')))"; done
