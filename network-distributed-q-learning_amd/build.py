"""Build the HIP library in-tree (and, for tests, the host build of the same kernel body).

Provenance: every build compiles the SHA-1 of its sources in (``SFL_BUILD_ID``, exported as
``sfl_build_id()`` and present in the file as the marker ``SFL_BUILD_ID:<sha1>``).  A library whose
marker differs from the sources in the tree is stale: ``build_hip`` / ``build_hostsim`` rebuild it,
and ``_lib.load_product`` refuses to run one.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SFL_ARCH", "gfx950")
SOURCES = ["sfl.hip", "sfl_core.h", "sfl_wave.h", "sfl_rng.h", "sfl_engine.h", "sfl_part.h", "sfl_mfgen.h", "sfl_capi.inc", "sfl_hostsim.cpp",
           os.path.join("..", "..", "include", "sfl.h")]
_MARK = re.compile(rb"SFL_BUILD_ID:([0-9a-f]{40})")


def kernel_source_sha1() -> str:
    """Hash of every source the libraries are built from: compiled into them as the build id, and ties a
    committed profile (profiles/*_pmc.json) to the kernel it measured."""
    h = hashlib.sha1()
    for f in SOURCES:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()


def built_id(path: str):
    """The build id compiled into a library file (None: missing, or built without one)."""
    if not os.path.exists(path):
        return None
    m = _MARK.search(open(path, "rb").read())
    return m.group(1).decode() if m else None


def _stale(out: str) -> bool:
    return built_id(out) != kernel_source_sha1()


def build_hip(force: bool = False, verbose: bool = False, out: str = None, defines=(), flags=()) -> str:
    """hipcc build of libsfl.so (gfx950).  ``out``/``defines``/``flags``: alternative builds for tuning."""
    out = os.path.abspath(out or os.path.join(HERE, "libsfl.so"))
    if force or _stale(out):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               "-Wno-unused-result", "-Wno-unused-value", f'-DSFL_BUILD_ID="{kernel_source_sha1()}"'] + \
              [f"-D{d}" for d in defines] + list(flags) + ["-o", out + ".tmp", os.path.join(CSRC, "sfl.hip")]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(out + ".tmp", out)
    return out


def build_hostsim(out_dir: str = None, force: bool = False) -> str:
    """The same kernel body compiled for the host CPU (libsfl_hostsim.so, OpenMP over envs): the
    parity tests' host build and bench.py's C++ CPU baseline -- never the product path.  Built
    in-tree so that it travels to the GPU box with the snapshot."""
    out_dir = out_dir or HERE
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.abspath(os.path.join(out_dir, "libsfl_hostsim.so"))
    if force or _stale(out):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fopenmp",
               f'-DSFL_BUILD_ID="{kernel_source_sha1()}"', "-o", out + ".tmp", os.path.join(CSRC, "sfl_hostsim.cpp")]
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_hip(force="--force" in sys.argv, verbose=True))
