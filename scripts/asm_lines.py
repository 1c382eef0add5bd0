"""Static instruction attribution of one kernel in a `hipcc -g -S` listing: instruction counts by
class (SALU / VALU / SMEM / VMEM / LDS / branch) per source line, for finding which source lines
feed the scalar and vector pipes.  Usage: python scripts/asm_lines.py listing.s KERNEL_SUBSTR [file]"""
import collections
import re
import sys


def classify(op):
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_endpgm", "s_barrier", "s_setprio", "s_sleep"):
        return None
    if op.startswith("s_cbranch") or op.startswith("s_branch") or op.startswith("s_setpc") or op.startswith("s_swappc"):
        return "BR"
    if op.startswith("s_load") or op.startswith("s_buffer_load") or op.startswith("s_memtime"):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    return None


def main(path, kern, only=None):
    files = {}
    cur = None
    inside = False
    cnt = collections.defaultdict(collections.Counter)
    for line in open(path):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", line)
        if m:
            files[m.group(1)] = m.group(2)
            continue
        if re.match(r"^_Z\S*:", line):
            inside = kern in line
            continue
        if not inside:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
            inside = False
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        m = re.match(r"\s+([a-z_0-9]+)", line)
        if m and cur:
            c = classify(m.group(1))
            if c:
                cnt[cur][c] += 1
    tot = collections.Counter()
    for k, v in sorted(cnt.items()):
        tot.update(v)
        if only and k[0] != only:
            continue
        print(f"{k[0]}:{k[1]:5d}  " + " ".join(f"{c}={n}" for c, n in sorted(v.items())))
    print("TOTAL", dict(tot))


if __name__ == "__main__":
    main(*sys.argv[1:])
