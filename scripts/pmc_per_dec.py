"""Per-decision (agent-env-step) instruction and cycle counts of the env kernel from one rocprofv3 --pmc
pass of bench.py (median over launches after the first).  Usage: python scripts/pmc_per_dec.py DIR [decisions]"""
import csv
import glob
import os
import statistics
import sys

src = sys.argv[1]
dec = float(sys.argv[2]) if len(sys.argv) > 2 else 65536 * 1024  # bench.py default launch: 65,536 envs x 1024 decisions
vals = {}
files = []
for d in glob.glob(src):  # a directory, or a glob of several (one per PMC pass)
    files += glob.glob(os.path.join(d, "*counter_collection.csv")) + glob.glob(os.path.join(d, "*", "*counter_collection.csv"))
for f in files:
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Kernel_Name"] or "k_wave" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k][1:] if len(vals[k]) > 1 else vals[k]
    print(f"{k:32s} per-decision {statistics.median(v) / dec:11.2f}   per launch {statistics.median(v):.4g}")
