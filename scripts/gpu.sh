# The one GPU launcher (replaces the per-round scripts/gpu_r*.sh): run the named steps in order on the gpurun box,
# each under its own time limit, stopping at the first failure.  Outputs under gpurun_out/$TAG.
#
#   gpurun --timeout 1200 -- 'TAG=r6a bash scripts/gpu.sh tests smoke bench'
#
# Steps:
#   tests      pytest -m gpu (PYTEST_K: a -k filter)
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (CPU baselines, oracle parity); BENCH_ARGS appended
#   driver     the driver's own command: bench.py --steps 20 --warmup 5
#   ktrace     rocprofv3 --kernel-trace --stats of a short bench (BENCH_ARGS)
#   pmc        the HBM-traffic passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss, memory-side requests) of a short bench
#   waitsplit  the wave-time split per decision (scripts/pmc_per_dec.py; DEC = decisions per launch)
#   final      the committed build's evidence: ktrace + traffic passes + waitsplit, summarised into
#              profiles/$PTAG_pmc.json on the box, THEN the default and the driver-style bench lines (which attach it)
#   c2         the same for configs[1] (c2 at its 4,096 envs): profiles/$PTAG_c2_4096_pmc.json, then its bench line
#   c2dec      configs[1] at 1,024 / 4,096 / 16,384 decisions per env and launch (C2DEC)
#   c2big      c2 at 65,536 envs
#   c5fused    c5 fused at 16,384 envs
#   part       the 8-rank partition rehearsal on one GPU (with the env-sharded fused comparison)
#   partrccl   the same with the segments exchanged by RCCL all-to-alls of a one-rank group
#   ab         bench for each library in LIBS (SFL_LIB, --experimental for all but libsfl)
#   rehearse   bench.py --gpus 2 / 4 (REH_N) as gloo ranks sharing this GPU: launcher, sharding, parity, the leg
#   abenv      bench of the product library for each runtime setting in ABENV (e.g. "SFL_LDS_MAP=1 SFL_LDS_MAP=0")
#   eval       the published evaluation table (scripts/eval_table.py) through libsfl.so, 15 trains
#   eval100    one 100-train learning run + greedy evaluation through libsfl.so (SEEDS100, default 66)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gpu}
mkdir -p $OUT

ok() { local rc=$1; shift; echo "$* rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
line() { python -c "import json,sys;d=json.load(open('$1'));r=d.get('roofline') or {};print('  %s %.1fM/s %.2f ms/step kernel %s ms frac %s parity %s' % ('$1'.split('/')[-1], d['value']/1e6, d['ms_per_step'], r.get('avg_kernel_ms'), r.get('frac'), d.get('parity')))"; }
SHORT="--no-cpu --sustain-seconds 0 --verify-envs 0"

ktrace() {  # ktrace <dir> <bench args...>
  local d=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o ktrace --output-format csv -- python bench.py --steps 10 --warmup 2 $SHORT "$@" > $d.json 2>/dev/null
}
pmc() {  # pmc <dir> <bench args...>: one --pmc pass per counter group
  local d=$1; shift
  for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" "TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ_ATOMIC_DRAM_32B TCC_EA0_WRREQ"; do
    local N=$(echo $C | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $d/pmc_$N -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 $SHORT "$@" > /dev/null 2>&1
    ok $? "pmc $N"
  done
}

for S in "$@"; do
  case $S in
    tests)
      timeout -k 10 1100 python -u -m pytest tests/test_gpu.py -x -v --durations=30 --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; ok $rc "tests" ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; ok $rc "smoke" ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/bench.err; ok $rc "bench"; line $OUT/bench.json ;;
    driver)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/driver.json 2> $OUT/driver.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/driver.err; ok $rc "driver"; line $OUT/driver.json ;;
    ktrace)
      ktrace $OUT/prof ${BENCH_ARGS}; ok $? "ktrace" ;;
    pmc)
      pmc $OUT ${BENCH_ARGS} ;;
    waitsplit)
      TAG=${TAG:-gpu} bash scripts/gpu_waitsplit.sh; ok $? "waitsplit" ;;
    final)  # the committed build's evidence: kernel stats, traffic passes, wave-time split, their summary as
            # profiles/${PTAG}_pmc.json (bench.py attaches it by build id), then the default and the driver's bench lines
      P=${PTAG:-${TAG:-gpu}}
      ktrace $OUT/prof; ok $? "ktrace"
      pmc $OUT
      TAG=${TAG:-gpu} bash scripts/gpu_waitsplit.sh > $OUT/waitsplit.log; ok $? "waitsplit"
      python scripts/pmc_summary.py $OUT profiles/${P}_pmc.json $OUT/prof.json > $OUT/pmc_summary.log; ok $? "pmc summary"
      cp profiles/${P}_pmc.json $OUT/
      timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/bench.err; ok $rc "bench"; line $OUT/bench.json
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/driver.json 2> $OUT/driver.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/driver.err; ok $rc "driver"; line $OUT/driver.json ;;
    c2)
      P=${PTAG:-${TAG:-gpu}}
      B="--config c2 --envs 4096"
      ktrace $OUT/c2_prof $B; ok $? "c2 ktrace"
      pmc $OUT/c2 $B
      TAG=${TAG:-gpu}/c2 BENCH_ARGS="$B --verify-envs 0" DEC=$((4096*1024)) bash scripts/gpu_waitsplit.sh > $OUT/c2_waitsplit.log; ok $? "c2 waitsplit"
      python scripts/pmc_summary.py $OUT/c2 profiles/${P}_c2_4096_pmc.json $OUT/c2_prof.json > $OUT/c2_pmc_summary.log; ok $? "c2 pmc summary"
      cp profiles/${P}_c2_4096_pmc.json $OUT/
      timeout -k 10 300 python bench.py $B --steps 10 --warmup 2 --no-cpu > $OUT/c2_bench.json 2> $OUT/c2_bench.err; ok $? "c2 bench"
      line $OUT/c2_bench.json ;;
    c2dec)  # configs[1] at longer launches (decisions per env per step): does the one-generation tail amortise?
      for D in ${C2DEC:-1024 4096 16384}; do
        timeout -k 10 300 python bench.py --config c2 --envs 4096 --decisions $D --steps $((10240 / D > 2 ? 10240 / D : 2)) --warmup 1 $SHORT > $OUT/c2_dec$D.json 2> $OUT/c2_dec$D.err; ok $? "c2 decisions $D"
        line $OUT/c2_dec$D.json
      done ;;
    c2big)
      timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu > $OUT/c2_65536_bench.json 2> $OUT/c2_65536.err; ok $? "c2 65536"
      line $OUT/c2_65536_bench.json ;;
    c5fused)
      timeout -k 10 300 python bench.py --config c5 --envs 16384 --steps 4 --warmup 1 --no-cpu > $OUT/c5_fused_bench.json 2> $OUT/c5_fused.err; ok $? "c5 fused"
      line $OUT/c5_fused_bench.json ;;
    part)
      timeout -k 10 400 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8 --verify-envs 4 ${PART_ARGS} > $OUT/part.json 2> $OUT/part.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/part.err; ok $rc "part"
      line $OUT/part.json
      python -c "import json;d=json.load(open('$OUT/part.json'));print('  fused env-sharded %.1fM/s, vs_env_sharded_fused %.3f' % (d['env_sharded_fused']['value']/1e6, d['vs_env_sharded_fused']))" ;;
    partrccl)  # the partition rehearsal with its segments as RCCL collectives of a one-rank group (RCCL's round cost)
      timeout -k 10 400 python bench.py --partition --steps 3 --warmup 1 --decisions 1024 --virtual-ranks 8 --verify-envs 4 --rccl-one-rank ${PART_ARGS} > $OUT/part_rccl.json 2> $OUT/part_rccl.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/part_rccl.err; ok $rc "part rccl"
      line $OUT/part_rccl.json
      python -c "import json;d=json.load(open('$OUT/part_rccl.json'));c=d['config'];print('  exchange %s, %s collectives/round, %.1f rounds/step, cohorts %s' % (c['exchange'], c['collectives_per_round'], c['rounds_per_step'], c['cohorts']))" ;;
    ab)
      i=0
      for L in ${LIBS:-libsfl}; do
        i=$((i+1))
        export SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so
        V="--verify-envs ${VERIFY_ENVS:-0} --experimental"; [ "$L" = "libsfl" ] && V=""
        timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu --sustain-seconds 0 $V ${BENCH_ARGS} > $OUT/ab_${i}_${L}.json 2> $OUT/ab_${i}_${L}.err; ok $? "ab $L"
        line $OUT/ab_${i}_${L}.json
      done
      unset SFL_LIB ;;
    rehearse)  # the N > 1 bench path on this one GPU: REH_N gloo ranks sharing device 0 (not the RCCL transport)
      for N in ${REH_N:-2 4}; do
        SFL_DIST_BACKEND=gloo SFL_DEVICE=0 timeout -k 10 600 python bench.py --gpus $N --envs 8192 --steps 3 --warmup 1 > $OUT/gpus$N.json 2> $OUT/gpus$N.err; rc=$?
        [ $rc -eq 0 ] || tail -5 $OUT/gpus$N.err; ok $rc "rehearse --gpus $N"
        python -c "import json;d=json.loads([l for l in open('$OUT/gpus$N.json') if l.startswith('{')][0]);L=d.get('partition_leg') or {};print('  world %d %s %.1fM/s parity %s (%d envs, %d threads/rank); leg %s parity %s vs fused %s' % (d['world_size'], d['backend'], d['value']/1e6, d['parity'], d['parity_envs_checked'], d['parity_threads_per_rank'], L.get('value'), L.get('parity'), L.get('vs_env_sharded_fused')))"
      done ;;
    abenv)  # the product library under each runtime setting in ABENV (e.g. "SFL_LDS_MAP=1 SFL_LDS_MAP=0"), BENCH_ARGS
      i=0
      for E in ${ABENV}; do
        i=$((i+1))
        N=$(echo $E | tr '=' '_')
        env $E timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu --sustain-seconds 0 ${BENCH_ARGS} > $OUT/abenv_${i}_${N}.json 2> $OUT/abenv_${i}_${N}.err; ok $? "abenv $E"
        line $OUT/abenv_${i}_${N}.json
      done ;;
    eval)  # the 15-train sweep config with malfunctions, 3 seeds x 10 evaluations, vs the host build's run
      timeout -k 10 900 python -u scripts/eval_table.py $OUT/eval_table.json --compare profiles/r06_eval_table_host.json ${EVAL_ARGS} > $OUT/eval_table.log 2>&1; rc=$?
      grep -v "^\.\.\." $OUT/eval_table.log | tail -6; ok $rc "eval" ;;
    eval100)  # one 100-train learning run (the two-slot k_wave shape) vs the host build's run of the same seed
      timeout -k 10 1000 python -u scripts/eval_table.py $OUT/eval100.json --trains 100 --size 100 --cities 25 --mf 0,0,0 --seeds ${SEEDS100:-66} --compare profiles/r06_100_trains_host.json > $OUT/eval100.log 2>&1; rc=$?
      grep -v "^\.\.\." $OUT/eval100.log | tail -6; ok $rc "eval100" ;;
    *)
      echo "unknown step $S"; exit 2 ;;
  esac
done
