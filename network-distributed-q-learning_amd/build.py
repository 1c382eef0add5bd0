"""Build the HIP library in-tree (and, for tests, the host build of the same kernel body)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SFL_ARCH", "gfx950")
SOURCES = ["sfl.hip", "sfl_core.h", "sfl_wave.h", "sfl_rng.h", "sfl_engine.h", "sfl_part.h", "sfl_capi.inc", "sfl_hostsim.cpp",
           os.path.join("..", "..", "include", "sfl.h")]


def kernel_source_sha1() -> str:
    """Hash of the device-code sources: ties a committed profile (profiles/*_pmc.json) to the kernel it measured."""
    import hashlib
    h = hashlib.sha1()
    for f in ("sfl.hip", "sfl_core.h", "sfl_wave.h", "sfl_rng.h"):
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()


def _stale(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(os.path.join(CSRC, s)) > t for s in srcs)


def build_hip(force: bool = False, verbose: bool = False, out: str = None, defines=(), flags=()) -> str:
    """hipcc build of libsfl.so (gfx950).  ``out``/``defines``/``flags``: alternative builds for tuning."""
    out = os.path.abspath(out or os.path.join(HERE, "libsfl.so"))
    if force or _stale(out, SOURCES):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               "-Wno-unused-result", "-Wno-unused-value"] + [f"-D{d}" for d in defines] + list(flags) + [
               "-o", out + ".tmp", os.path.join(CSRC, "sfl.hip")]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(out + ".tmp", out)
    return out


def build_hostsim(out_dir: str = None, force: bool = False) -> str:
    """The same kernel body compiled for the host CPU (libsfl_hostsim.so, OpenMP over envs): the
    parity tests' host build and bench.py's C++ CPU baseline leg -- never the product path.  Built
    in-tree so that it travels to the GPU box with the snapshot."""
    out_dir = out_dir or HERE
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.abspath(os.path.join(out_dir, "libsfl_hostsim.so"))
    if force or _stale(out, SOURCES):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fopenmp",
               "-o", out + ".tmp", os.path.join(CSRC, "sfl_hostsim.cpp")]
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_hip(force="--force" in sys.argv, verbose=True))
