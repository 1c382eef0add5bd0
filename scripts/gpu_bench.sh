set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
echo "== rocprof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; echo "prof rc=$?"
find gpurun_out/prof -name "*stats*" | head; 
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat $f; done
