# round 4 (f): the product after the epsilon A/B (table load kept) and the early reply load: GPU suite, default
# bench with the CPU baselines, c2 at 65,536 and 4,096 envs, the partition rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r4f STEPS="tests" bash scripts/gpu_r4.sh || exit 1
mkdir -p gpurun_out/r4f
timeout -k 10 600 python bench.py > gpurun_out/r4f/bench_default.json 2> gpurun_out/r4f/bench_default.err; rc=$?; echo "default bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/r4f/bench_default.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/r4f/bench_default.json'));print('  %.1fM/s kernel %.3f ms parity %s cpu %s' % (d['value']/1e6, d['roofline']['avg_kernel_ms'], d.get('parity'), d.get('cpu_baseline',{}).get('value')))"
TAG=r4f_c2 STEPS="bench" BENCH_ARGS="--config c2" bash scripts/gpu_r4.sh || exit 1
TAG=r4f_c2_4096 STEPS="bench" BENCH_ARGS="--config c2 --envs 4096" bash scripts/gpu_r4.sh || exit 1
TAG=r4f STEPS="part" bash scripts/gpu_r4.sh
