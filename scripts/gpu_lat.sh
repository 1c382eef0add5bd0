# Memory latency / translation counters (one rocprofv3 --pmc pass each) for LIBS x GS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lat}
mkdir -p $OUT
for L in ${LIBS:-libsfl}; do
  for g in ${GS:-64}; do
    export SFL_LIB=$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/$L.so SFL_WAVE_G=$g
    i=0
    for C in VmemLatency SmemLatency LdsLatency "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/lat_${L}_g${g}_$i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "pmc $L G=$g pass $i ($C) rc=$rc"; exit $rc; }
    done
    echo "== $L G=$g"
    python scripts/pmc_per_dec.py "$OUT/lat_${L}_g${g}_*" | sed 's/^/  /'
  done
done
