"""Per-kernel per-launch medians of the PMC passes of scripts/gpu_c5pmc.sh (the partitioned round's kernels), as
the JSON committed under profiles/ (e.g. r03_c5_virtual8_pmc_per_kernel.json).  Usage:
python scripts/pmc_per_kernel.py gpurun_out/<tag> profiles/<name>.json [envs]"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def main(src, dst, envs=16384):
    vals = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {"workload": "bench.py --partition --virtual-ranks 8 --decisions 128 --steps 1 --warmup 1 (c5, %d envs, one rank)"
                       % envs,
           "note": "per-launch medians; FETCH_SIZE / WRITE_SIZE in KiB (FETCH x2 on gfx950 for 128-B requests); SQ_* in "
                   "quad-cycles / instructions summed over waves; *_per_env = per local-step launch / envs",
           "kernels": {}}
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        for c in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD"):
            if c in med and ("wave" in k or "part_local" in k):
                med[c + "_per_env"] = med[c] / envs
        out["kernels"][k] = med
    json.dump(out, open(dst, "w"), indent=1)
    for k, med in out["kernels"].items():
        print(k, {c: round(v, 1) for c, v in med.items() if c.endswith("_per_env")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 16384)
