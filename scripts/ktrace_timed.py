"""Average duration of the env kernel over the timed launches of a rocprofv3 --kernel-trace run of bench.py
(skipping the warm-up launches), to set beside the bench line's HIP-event average.
Usage: python scripts/ktrace_timed.py gpurun_out/<tag>/prof/ktrace_kernel_trace.csv [warmup]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_wave" in r["Kernel_Name"] or "k_run" in r["Kernel_Name"]]
w = int(sys.argv[2]) if len(sys.argv) > 2 else 2
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(f"{rows[0]['Kernel_Name'][:60]}: {len(d)} launches, timed average {sum(d[w:]) / len(d[w:]):.4f} ms "
      f"(all {sum(d) / len(d):.4f} ms)")
