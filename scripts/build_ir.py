"""Tuning builds of libsfl.so through the device LLVM IR, to set the register-file split of the grouped
kernels (k_wave_g): clang's attributor marks every kernel "amdgpu-agpr-alloc"="0" (no accumulation
registers), so at 4 waves per SIMD all 128 registers of a lane are architectural VGPRs and the
allocator spills to scratch memory.  With "amdgpu-agpr-alloc"="N" the unified file is split into
128 - N VGPRs + N AGPRs and spills go to the AGPRs first (v_accvgpr_write / read, no memory round trip).

The steps are hipcc's own, with the attribute edited in between: device bitcode (hipcc --cuda-device-only
-emit-llvm), llvm-dis, the edit, opt (assemble), lld LTO codegen (-amdgpu-internalize-symbols, O3, as
hipcc links), clang-offload-bundler, and the host side (hipcc --cuda-host-only with the bundle included).
The library carries the build id of its sources with the define SFL_AGPR_ALLOC=N (build.build_id), so
bench.py accepts it only with --experimental and names the define in its JSON line.

Usage: python scripts/build_ir.py N [N ...]   -> network-distributed-q-learning_amd/libsfl_agprN.so
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKGDIR = os.path.join(ROOT, "network-distributed-q-learning_amd")
sys.path.insert(0, PKGDIR)
import build  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "k_wave_g"


def set_agpr_alloc(ll: str, n: int, kernel: str = KERNEL) -> str:
    """Set "amdgpu-agpr-alloc"="n" in the attribute groups of the kernels whose name contains `kernel`
    (refused if such a group is shared with another function)."""
    groups, others = set(), set()
    for line in ll.splitlines():
        if line.startswith("define "):
            m = re.search(r"#(\d+)[^#]*\{\s*$", line)
            if not m:
                continue
            (groups if kernel in line.split("(")[0] else others).add(m.group(1))
    if groups & others:
        raise SystemExit(f"attribute groups {groups & others} are shared with other functions")
    out = []
    for line in ll.splitlines():
        m = re.match(r"attributes #(\d+) = \{", line)
        if m and m.group(1) in groups:
            if '"amdgpu-agpr-alloc"' in line:
                line = re.sub(r'"amdgpu-agpr-alloc"="[^"]*"', f'"amdgpu-agpr-alloc"="{n}"', line)
            else:
                line = line.replace("{", f'{{ "amdgpu-agpr-alloc"="{n}"', 1)
        out.append(line)
    return "\n".join(out) + "\n"


def build_agpr(n: int, out: str = None, extra=()) -> str:
    defines = [f"SFL_AGPR_ALLOC={n}"] + list(extra)
    out = out or os.path.join(PKGDIR, f"libsfl_agpr{n}.so")
    src = os.path.join(build.CSRC, "sfl.hip")
    common = ["-O3", "-std=c++17", "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-value",
              f'-DSFL_BUILD_ID="{build.build_id(defines)}"', f'-DSFL_BUILD_DEFS="{" ".join(defines)}"'] + \
             [f"-D{d}" for d in defines]
    with tempfile.TemporaryDirectory() as tmp:
        p = lambda x: os.path.join(tmp, x)  # noqa: E731
        run = lambda cmd: subprocess.run(cmd, check=True, cwd=build.CSRC)  # noqa: E731
        run([build.HIPCC, f"--offload-arch={build.ARCH}", "--cuda-device-only", "-emit-llvm", "-c"] + common +
            ["-o", p("dev.bc"), src])
        run([f"{LLVM}/llvm-dis", p("dev.bc"), "-o", p("dev.ll")])
        open(p("dev2.ll"), "w").write(set_agpr_alloc(open(p("dev.ll")).read(), n))
        run([f"{LLVM}/opt", p("dev2.ll"), "-o", p("dev2.bc")])  # (no passes: assemble only)
        run([f"{LLVM}/lld", "-flavor", "gnu", "-m", "elf64_amdgpu", "--no-undefined", "-shared",
             "-plugin-opt=-amdgpu-internalize-symbols", "--lto-partitions=8", f"-plugin-opt=mcpu={build.ARCH}",
             # (the LTO pipeline would run the attributor again and re-infer "amdgpu-agpr-alloc"="0"; the
             # pre-link pipeline already ran it, so its other inferences are in the bitcode)
             "-plugin-opt=-amdgpu-attributor-enable=0",
             "-plugin-opt=O3", "--lto-CGO3", "-o", p("dev.hsaco"), p("dev2.bc")])
        run([f"{LLVM}/clang-offload-bundler", "-type=o", "-bundle-align=4096",
             f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{build.ARCH}", "-input=/dev/null",
             f"-input={p('dev.hsaco')}", f"-output={p('dev.hipfb')}"])
        run([build.HIPCC, f"--offload-arch={build.ARCH}", "--cuda-host-only", "-fPIC", "-shared"] + common +
            ["-Xclang", "-fcuda-include-gpubinary", "-Xclang", p("dev.hipfb"), "-o", out + ".tmp", src])
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # python scripts/build_ir.py N [OUT.so DEFINE ...]: one build with extra tuning defines
    if len(sys.argv) > 2 and sys.argv[2].endswith(".so"):
        print(build_agpr(int(sys.argv[1]), os.path.join(PKGDIR, sys.argv[2]), sys.argv[3:]))
    else:
        for a in sys.argv[1:]:
            print(build_agpr(int(a)))
