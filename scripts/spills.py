"""Scratch (spill) instructions of one kernel in a `hipcc -S -gline-tables-only` listing, by source line.
Usage: python scripts/spills.py listing.s [KERNEL_SUBSTR]   (default: the c3 bench kernel, k_wave_g variant 7)"""
import collections
import re
import sys

path = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_wave_gILi16ELi4ELi32ELb0ELi16ELi4ELb0E"
txt = open(path).read()
files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
         for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]+)"(?:\s+"([^"]+)")?', txt)}
name = next(m.group(1) for m in re.finditer(r"^([^\s:]+):", txt, re.M) if kern in m.group(1) and not m.group(1).startswith("."))
body = txt[txt.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
cur, cnt, tot = None, collections.Counter(), collections.Counter()
for line in body.splitlines():
    s = line.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    if not s or s.startswith((".", ";")) or s.endswith(":"):
        continue
    op = s.split()[0]
    tot["instructions"] += 1
    tot["valu"] += op.startswith("v_")
    if op.startswith("scratch_"):
        cnt[(cur, op.split("_")[1])] += 1
print(f"{name}: {tot['instructions']} instructions, {tot['valu']} VALU, {sum(cnt.values())} scratch")
for (loc, kind), c in sorted(cnt.items(), key=lambda x: (x[0][0] or "", x[0][1])):
    print(f"  {loc:24s} {kind:5s} {c}")
