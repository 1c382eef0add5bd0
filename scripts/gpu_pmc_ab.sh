# Instruction mix per decision (rocprofv3 --pmc, two passes) for each library in LIBS x lane-group size in GS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcab}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  for g in ${GS:-64}; do
    export SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so SFL_WAVE_G=$g
    P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
    P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
    i=0
    for C in "$P1" "$P2"; do
      i=$((i+1))
      timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${L}_g${g}_$i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "pmc $L G=$g pass $i rc=$rc"; exit $rc; }
    done
    echo "== $L G=$g"
    python scripts/pmc_per_dec.py "$OUT/pmc_${L}_g${g}_*" | sed 's/^/  /'
  done
done
