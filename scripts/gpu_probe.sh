set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
rocprofv3 -L > gpurun_out/probe/counters.txt 2>&1 || true
grep -i -E "utcl|tlb|TCP_TCC|TA_BUSY|TCC_EA0_RD|TCC_HIT|TCC_MISS|FETCH_SIZE|WRITE_SIZE|SQ_WAIT|SQ_WAVE_CYCLES|SQ_INSTS_VMEM|SQ_INSTS_VALU|MALL" gpurun_out/probe/counters.txt | head -80
for E in 4096 16384 65536; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --envs $E > gpurun_out/probe/bench_$E.json 2>/dev/null
  echo "E=$E rc=$?"; python -c "import json;d=json.load(open('gpurun_out/probe/bench_$E.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
done
