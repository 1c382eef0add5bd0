# PC sampling of the env kernel (statistical per-instruction profile) on a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pcs}
mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -i -A3 "pc.sampl\|PC_SAMPL\|method" $OUT/avail.txt | head -40
SFL_LIB=${SFL_LIB:-$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_g.so} timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-host_trap} --pc-sampling-unit ${UNIT:-time} --pc-sampling-interval ${INTERVAL:-1} -d $OUT/pcs -o pcs --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "pcs rc=$rc"; ls -la $OUT/pcs/* 2>/dev/null | head; tail -5 $OUT/bench.err
exit $rc
