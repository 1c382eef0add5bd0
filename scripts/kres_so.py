"""Kernel resource usage (VGPRs, spills, LDS, scratch) of the gfx950 code object inside a built libsfl*.so:
the offload bundle is cut out of the library and its AMDGPU metadata note read with llvm-readelf.
Usage: python scripts/kres_so.py LIB.so [KERNEL_SUBSTR]"""
import re
import struct
import subprocess
import sys
import tempfile


def code_object(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    i = data.find(magic)
    n = struct.unpack_from("<Q", data, i + len(magic))[0]
    p = i + len(magic) + 8
    for _ in range(n):
        off, size, idlen = struct.unpack_from("<QQQ", data, p)
        tid = data[p + 24:p + 24 + idlen].decode()
        p += 24 + idlen
        if "gfx950" in tid:
            return data[i + off:i + off + size]
    raise SystemExit("no gfx950 code object in " + path)


def main(path, sub="k_wave_g"):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object(path))
        f.flush()
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name], capture_output=True,
                               text=True).stdout
    for blk in notes.split("- .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if sub not in name:
            continue
        g = lambda k: re.search(r"\." + k + r":\s+(\d+)", blk).group(1)
        agpr = blk.split()[0]
        print(f"{name[:90]:90s} agpr {agpr:>3s} vgpr {g('vgpr_count'):>3s} vspill {g('vgpr_spill_count'):>3s} "
              f"sspill {g('sgpr_spill_count'):>3s} lds {g('group_segment_fixed_size'):>6s} "
              f"scratch {g('private_segment_fixed_size'):>4s}")


if __name__ == "__main__":
    main(*sys.argv[1:])
