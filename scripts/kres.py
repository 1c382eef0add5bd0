"""Per-kernel VGPRs / scratch / occupancy of libsfl's device code (hipcc -Rpass-analysis=kernel-resource-usage).
Usage: python scripts/kres.py [extra hipcc -D flags...]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-result",
       "-Wno-unused-value", "--offload-device-only", "-c", "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/kres.o",
       "network-distributed-q-learning_amd/csrc/sfl.hip"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    for key, pat in (("V", r"VGPRs: (\d+)"), ("A", r"AGPRs: (\d+)"), ("scr", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            rows[cur][key] = int(m.group(1))
for name, r in rows.items():
    if "k_wave" not in name:
        continue
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name).split("EEEvPK")[0]
    print(f"{short:40s} " + " ".join(f"{k}={v}" for k, v in r.items()))
