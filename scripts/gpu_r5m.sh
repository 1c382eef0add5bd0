# round 5, call M: env cohorts for the partitioned round (partition.CohortPipeline): GPU partition tests,
# then the 8-rank rehearsal (c5, 16,384 envs, 1,024 decisions) with 1 / 2 / 3 / 4 cohorts on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5m}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "cohort or partition" > $OUT/pytest_part.log 2>&1; rc=$?
echo "pytest part rc=$rc"; tail -2 $OUT/pytest_part.log; [ $rc -eq 0 ] || exit $rc
fi
P="--partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8"
# COHORTS entries: <cohorts> or <cohorts>q<hardware queues> (GPU_MAX_HW_QUEUES for that run)
for CQ in ${COHORTS:-1 2 3 4 1 2}; do
  C=${CQ%q*}; Q=""; [ "$CQ" != "$C" ] && Q=${CQ#*q}
  if [ -n "$Q" ]; then export GPU_MAX_HW_QUEUES=$Q; else unset GPU_MAX_HW_QUEUES; fi
  timeout -k 10 300 python bench.py $P --verify-envs 4 --cohorts $C > $OUT/part_c$CQ.json 2> $OUT/part_c$CQ.err; rc=$?; echo "cohorts $CQ rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/part_c$CQ.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/part_c$CQ.json'));print('  %.1fM/s  %.1f ms/step  rounds/step %s parity %s' % (d['value']/1e6, d['ms_per_step'], d['config']['rounds_per_step'], d.get('parity')))"
done
