"""FETCH_SIZE / WRITE_SIZE calibration factors from rocprofv3 --pmc passes over scripts/calib/fetch_calib.bin.

Usage: python scripts/calib/fetch_calib.py gpurun_out/<tag> profiles/<name>.json
<tag> holds calib.json (the binary's own line: bytes and lines per launch of every kernel) and one
directory per counter pass (calib_<COUNTER>/ with rocprofv3's *counter_collection.csv).

Per kernel shape: the counter's bytes per launch (FETCH_SIZE / WRITE_SIZE are KiB) divided by the bytes
the lanes asked for, and by the 128-B lines they touched.  The factor the bench's traffic estimate needs is
`true bytes / counter bytes` for the access shape: for the scattered shapes no line is shared by two
accesses, so the bytes that must cross the memory interface are at least one memory request per access;
what the counter reports per access is printed so the reader can see which request size it tallies.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def load(tag):
    vals = {}
    for f in glob.glob(os.path.join(tag, "calib_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0]
            vals.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main(tag, dst):
    known = json.load(open(os.path.join(tag, "calib.json")))
    med = load(tag)
    out = {"table_bytes": known["table_bytes"], "accesses_per_launch": known["accesses_per_launch"], "kernels": {}}
    counters = sorted({c for (_, c) in med})
    for name, kb in known["kernels"].items():
        row = {"bytes_requested": kb["bytes"], "lines_touched": kb["lines"]}
        for c in counters:
            v = med.get((name, c))
            if v is None:
                continue
            row[c] = v
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                b = v * 1024.0
                row[c + "_bytes_per_request_byte"] = b / kb["bytes"]
                row[c + "_bytes_per_line"] = b / kb["lines"]
        out["kernels"][name] = row
    json.dump(out, open(dst, "w"), indent=1)
    w = max(len(n) for n in out["kernels"])
    for n, r in out["kernels"].items():
        print(f"{n:{w}s}  " + "  ".join(f"{k}={r[k]:.4g}" for k in r if k.endswith("_per_line") or k.endswith("_request_byte")))


if __name__ == "__main__":
    main(*sys.argv[1:3])
