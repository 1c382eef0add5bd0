# round 4, final: the evidence for the committed product build in one call -- GPU suite, smoke, default bench
# (CPU baselines, oracle parity), rocprofv3 kernel stats, the HBM-traffic PMC passes and the wave-time split of
# the bench kernel (bench.py attaches them by build id), c2 at 65,536 and 4,096 envs, the partition rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4z
mkdir -p $OUT
TAG=r4z STEPS="tests" bash scripts/gpu_r4.sh || exit 1
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "default bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('  %.1fM/s kernel %.3f ms parity %s cpu %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity'), d.get('cpu_baseline',{}).get('value')))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --verify-envs 0 > $OUT/prof_bench.json 2>/dev/null; rc=$?; echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$N -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=r4z bash scripts/gpu_waitsplit.sh || exit 1
TAG=r4z_c2 STEPS="bench" BENCH_ARGS="--config c2" bash scripts/gpu_r4.sh || exit 1
TAG=r4z_c2_4096 STEPS="bench" BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh || exit 1
TAG=r4z STEPS="part" bash scripts/gpu_r4.sh
