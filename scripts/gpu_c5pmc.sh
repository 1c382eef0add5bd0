# C5 local step: HBM traffic and wave-time split of the partitioned round's kernels (one rocprofv3 --pmc pass
# per counter group) on the 8-rank rehearsal, 128 decisions per env.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c5pmc}
mkdir -p $OUT
i=0
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$i -o pmc --output-format csv -- python bench.py --partition --steps 1 --warmup 1 --decisions 128 --verify-envs 0 --virtual-ranks 8 ${BENCH_ARGS} > $OUT/pmc_$i.json 2>$OUT/pmc_$i.err
  rc=$?; echo "pmc $i ($C) rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/pmc_$i.err; exit $rc; }
done
