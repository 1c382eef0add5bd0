# round 5, final evidence for the committed build (part 1): GPU suite, smoke, default bench (CPU baselines, oracle
# parity), rocprofv3 kernel stats, HBM-traffic PMC passes (incl. the memory-side request counters) and the wave-time
# split of the bench kernel (bench.py attaches them by build id).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5z}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "default bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('  %.1fM/s kernel %.3f ms parity %s cpu %s oracle %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_oracle_baseline',{}).get('value')))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --sustain-seconds 0 --verify-envs 0 > $OUT/prof_bench.json 2>/dev/null; rc=$?; echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" "TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ_ATOMIC_DRAM_32B TCC_EA0_WRREQ"; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$N -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --sustain-seconds 0 --verify-envs 0 > /dev/null 2>&1; rc=$?; echo "pmc $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG:-r5z} bash scripts/gpu_waitsplit.sh || exit 1
