# Split the env kernel's wave time by source (round-3 verdict item 1, "measure first"): one rocprofv3
# --pmc pass per counter group on a short bench, then scripts/pmc_per_dec.py per decision.
#   pass 1: wave cycles, waits (any / issue / LDS issue), LDS instructions and bank conflicts
#   pass 2: VALU lane utilisation (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU)
#   pass 3-5: LDS / VMEM / SMEM latency (accumulated in-flight levels / instructions)
#   pass 6: instruction mix
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ws}
mkdir -p $OUT
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU" \
         LdsLatency VmemLatency SmemLatency \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $OUT/ws_$i -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --sustain-seconds 0 ${BENCH_ARGS} > $OUT/ws_$i.json 2>$OUT/ws_$i.err
  rc=$?; echo "pmc $i ($C) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_per_dec.py "$OUT/ws_*" ${DEC} > $OUT/per_dec.txt; cat $OUT/per_dec.txt
