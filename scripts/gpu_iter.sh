# Development iteration: GPU parity tests, bench, and the SQ instruction-mix PMC pass of the env kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/bench.json'));print('%.1fM/s kernel %.3f ms frac %.4f' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d['roofline']['frac']))"
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $OUT/pmc_mix -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS} > /dev/null 2>&1; rc=$?; echo "pmc rc=$rc"
[ $rc -eq 0 ] || exit $rc
python scripts/pmc_per_dec.py $OUT/pmc_mix
