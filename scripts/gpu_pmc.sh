# PMC passes (one rocprofv3 run per counter group, kernel-trace only) on a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_LDS" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
         "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_MISSES" "SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM" \
         FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$i -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/pmc_$i.json 2>$OUT/pmc_$i.err
  rc=$?; echo "pmc $i ($C) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
