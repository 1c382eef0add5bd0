# PC sampling of the c3 bench kernel (rocprofv3 beta): where the wave's samples land, instruction by instruction
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pcs}
mkdir -p $OUT
M=${PCS_METHOD:-stochastic}
U=${PCS_UNIT:-cycles}
I=${PCS_INTERVAL:-65536}
SFL_LIB=${SFL_LIB:-$GRAFT_REPO_ROOT/network-distributed-q-learning_amd/libsfl_g.so} timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U --pc-sampling-interval $I --kernel-trace -d $OUT/pcs -o pcs --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --verify-envs 0 --experimental ${BENCH_ARGS} > $OUT/pcs_bench.json 2> $OUT/pcs.err; rc=$?
echo "pcs $M/$U/$I rc=$rc"; tail -3 $OUT/pcs.err; ls -la $OUT/pcs | head; exit $rc
