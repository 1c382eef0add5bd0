"""Summarise rocprofv3 PMC passes for the env kernel (k_run / k_wave) into a JSON (HBM traffic per launch, gfx950-corrected).

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 64 B per 128-B request, i.e. half the
bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM) — we apply that x2 correction and note
that other access widths are uncalibrated.
Usage: python scripts/pmc_summary.py gpurun_out/<tag> profiles/<name>.json [bench.json of the same workload]
The PMC passes run bench.py with its default workload; the bench line's config.workload is
recorded so that bench.py reports the traffic only for that workload.
"""
import csv
import glob
import importlib
import json
import os
import statistics
import sys


def main(src, dst, bench_json=None):
    vals = {}
    kname = None
    for d in sorted(glob.glob(os.path.join(src, "pmc_*")) + glob.glob(os.path.join(src, "ws_*"))):
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if "k_run" in r["Kernel_Name"] or "k_wave" in r["Kernel_Name"]:
                    kname = r["Kernel_Name"]
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: statistics.median(v[1:] if len(v) > 1 else v) for k, v in vals.items()}  # skip the warm-up launch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    build = importlib.import_module("network-distributed-q-learning_amd.build")
    out = {"kernel": kname, "per_launch_median": med,
           "fetch_bytes_corrected": 2 * med.get("FETCH_SIZE", 0) * 1024,
           "write_bytes": med.get("WRITE_SIZE", 0) * 1024,
           "source_sha1": build.kernel_source_sha1(),
           "note": "FETCH_SIZE x2 (gfx950 half-count of 128-B requests); uncalibrated for narrow scattered access"}
    out["traffic_bytes_per_launch"] = out["fetch_bytes_corrected"] + out["write_bytes"]
    if "TCC_HIT_sum" in med:
        out["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in med:
        out["wait_fraction"] = med.get("SQ_WAIT_ANY", 0) / med["SQ_WAVE_CYCLES"]
    if bench_json:
        bj = json.load(open(bench_json))
        out["workload"] = bj["config"]["workload"]
        # the build id of the library the passes ran (sources + defines + flags): bench.py attaches this
        # profile only to a run of exactly that build
        if "library" in bj:
            out["build_id"] = bj["library"]["build_id"]
            out["defines"] = bj["library"]["defines"]
        # VALU issue against the SIMDs' capacity: a wave64 VALU instruction takes 2 SIMD cycles (SIMD-32;
        # MI355X_MICROARCH.md cycle constants), 1,024 SIMDs at 2.4 GHz over the kernel's average duration
        ms = (bj.get("roofline") or {}).get("avg_kernel_ms")
        if ms and "SQ_INSTS_VALU" in med:
            out["valu_issue_frac"] = med["SQ_INSTS_VALU"] * 2.0 / (1024 * ms * 1e-3 * 2.4e9)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
