# Rehearsal of the driver's multi-GPU bench launch on a one-GPU box: torch.distributed.run with 2
# ranks on GPU 0 over gloo (launcher, env sharding, timing max / decision sum, rank-0 JSON line),
# for the env-sharded bench and the graph-partitioned mode.  Not a scaling measurement.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp SFL_DIST_BACKEND=gloo SFL_DEVICE=0
OUT=gpurun_out/${TAG:-multirank}
mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --envs 16384 --decisions 256 > $OUT/bench2.json 2> $OUT/bench2.err; rc=$?
echo "bench 2 ranks rc=$rc"; cat $OUT/bench2.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench2.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 2 --partition --steps 2 --warmup 1 --envs 1024 --decisions 8 > $OUT/part2.json 2> $OUT/part2.err; rc=$?
echo "partition 2 ranks rc=$rc"; cat $OUT/part2.json; [ $rc -eq 0 ] || { tail -20 $OUT/part2.err; exit $rc; }
