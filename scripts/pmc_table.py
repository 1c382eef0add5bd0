"""Print the per-launch median of every PMC counter collected by scripts/gpu_pmc.sh for the env kernel."""
import csv
import glob
import json
import os
import statistics
import sys

src = sys.argv[1]
vals = {}
for f in sorted(glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Kernel_Name"] or "k_wave" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
med = {k: statistics.median(v[1:] if len(v) > 1 else v) for k, v in vals.items()}
b = json.load(open(sorted(glob.glob(os.path.join(src, "pmc_*.json")))[0]))
dec = b["roofline"]["alg_bytes_per_launch"]  # placeholder to keep the keys visible
print(json.dumps({k: med[k] for k in sorted(med)}, indent=1))
print("bench:", json.dumps(b["roofline"]))
