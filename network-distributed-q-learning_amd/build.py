"""Build the HIP library in-tree (and, for tests, the host build of the same kernel body).

Provenance: every build compiles its build id in (``SFL_BUILD_ID``, exported as ``sfl_build_id()`` and
present in the file as the marker ``SFL_BUILD_ID:<sha1>``): the SHA-1 of its sources, of the ``-D``
defines and of the extra compiler flags (``build_id``).  The defines are in the file too
(``SFL_BUILD_DEFS:[...]``).  The product build is the one with no defines and no flags: a library whose
id differs from the tree's product id is stale or an experiment; ``build_hip`` / ``build_hostsim``
rebuild a stale one, and ``_lib.load_product`` refuses to run either (an experiment library only with
``SFL_EXPERIMENTAL=1``, which ``bench.py --experimental`` sets and reports).  Timing-only switches that
make results invalid (``SFL_X_*`` / ``SFL_AB_*``, csrc/sfl_experiment.h) are never built into the
product path.
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
SOURCES = ["sfl.hip", "sfl_kwave_v7.hip", "sfl_kwave_g.h", "sfl_core.h", "sfl_wave.h", "sfl_rng.h", "sfl_engine.h", "sfl_part.h",
           "sfl_mfgen.h", "sfl_capi.inc", "sfl_hostsim.cpp", "sfl_experiment.h", os.path.join("..", "..", "include", "sfl.h")]
# libsfl.so's translation units and the compiler flags each adds to the common ones: variant 7 of k_wave_g (the
# bench's c3 shape) with LLVM's register-minimising machine scheduler -- c3 +6.5 %, every other kernel loses with
# it (round 5, profiles/r05p_sched_strategy_ab.txt).  Part of the build id (kernel_source_sha1).
TUS = {"sfl.hip": [], "sfl_kwave_v7.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]}
_MARK = re.compile(rb"SFL_BUILD_ID:([0-9a-f]{40})")
_DEFS = re.compile(rb"SFL_BUILD_DEFS:\[([^\]\x00]*)\]")
_FLAGS = re.compile(rb"SFL_BUILD_FLAGS:\[([^\]\x00]*)\]")
PRODUCT_LIB = os.path.join(HERE, "libsfl.so")
# timing-only switches whose builds compute wrong results (csrc/sfl_experiment.h)
EXPERIMENT_PREFIXES = ("SFL_X_", "SFL_AB_")


def kernel_source_sha1() -> str:
    """Hash of every source the libraries are built from: compiled into them as the build id, and ties a
    committed profile (profiles/*_pmc.json) to the kernel it measured."""
    h = hashlib.sha1()
    for f in SOURCES:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(repr(sorted(TUS.items())).encode())
    return h.hexdigest()


def build_id(defines=(), flags=()) -> str:
    """The id a build of the tree's sources with these -D defines and extra flags carries (no defines and
    no flags: the product build)."""
    if not defines and not flags:
        return kernel_source_sha1()
    h = hashlib.sha1(kernel_source_sha1().encode())
    h.update(("\0D" + "\n".join(sorted(defines)) + "\0F" + " ".join(flags)).encode())
    return h.hexdigest()


def product_build_id() -> str:
    return build_id()


def built_defines(path: str):
    """The -D defines recorded in a library file ("" for none; None if it carries no record)."""
    if not os.path.exists(path):
        return None
    m = _DEFS.search(open(path, "rb").read())
    return m.group(1).decode() if m else None


def built_flags(path: str):
    """The extra compiler flags recorded in a library file ("" for none; None if it carries no record)."""
    if not os.path.exists(path):
        return None
    m = _FLAGS.search(open(path, "rb").read())
    return m.group(1).decode() if m else None


def built_id(path: str):
    """The build id compiled into a library file (None: missing, or built without one)."""
    if not os.path.exists(path):
        return None
    m = _MARK.search(open(path, "rb").read())
    return m.group(1).decode() if m else None


def _stale(out: str, defines=(), flags=()) -> bool:
    return built_id(out) != build_id(defines, flags)


def link_cmd(out: str, objs, flags=()):
    """hipcc's link line of libsfl.so: the caller's extra flags go to the link too (a build with link-relevant
    flags -- -fgpu-rdc, sanitizer, profiling or coverage flags, -Wl,... -- must link with them; its build id
    already claims them)."""
    return [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + list(flags) + ["-o", out] + list(objs)


def build_hip(force: bool = False, verbose: bool = False, out: str = None, defines=(), flags=()) -> str:
    """hipcc build of libsfl.so (gfx950).  ``out``/``defines``/``flags``: alternative builds for tuning,
    never into the product path (libsfl.so); an ``SFL_X_*`` / ``SFL_AB_*`` define makes an experiment
    build (results invalid, csrc/sfl_experiment.h)."""
    out = os.path.abspath(out or PRODUCT_LIB)
    defines, flags = list(defines), list(flags)
    if (defines or flags) and out == os.path.abspath(PRODUCT_LIB):
        raise ValueError(f"build_hip: defines {defines} / flags {flags} are not built into the product library {out}; "
                         "pass out= for a tuning or experiment build")
    if any(d.startswith(EXPERIMENT_PREFIXES) for d in defines) and "SFL_EXPERIMENT" not in defines:
        defines.append("SFL_EXPERIMENT")
    if force or _stale(out, defines, flags):
        defs = " ".join(sorted(defines))
        common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                  "-Wno-unused-result", "-Wno-unused-value", f'-DSFL_BUILD_ID="{build_id(defines, flags)}"',
                  f'-DSFL_BUILD_DEFS="{defs}"', f'-DSFL_BUILD_FLAGS="{" ".join(flags)}"'] + \
                 [f"-D{d}" for d in defines] + list(flags)
        tmp = out + f".{os.getpid()}.tmp"
        objs, procs = [], []
        for tu, tu_flags in TUS.items():
            # (a tuning build that picks its own scheduler strategy applies it to every unit)
            extra = [] if any("amdgpu-sched-strategy" in f for f in flags) else tu_flags
            obj = f"{tmp}.{os.path.splitext(tu)[0]}.o"
            cmd = common + extra + ["-c", "-o", obj, os.path.join(CSRC, tu)]
            if verbose:
                print(" ".join(cmd), flush=True)
            objs.append(obj)
            procs.append((cmd, subprocess.Popen(cmd, cwd=CSRC)))
        try:
            for cmd, p in procs:
                if p.wait() != 0:
                    raise subprocess.CalledProcessError(p.returncode, cmd)
            subprocess.run(link_cmd(tmp, objs, flags), check=True, cwd=CSRC)
        finally:
            for cmd, p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
            for o in objs:
                if os.path.exists(o):
                    os.remove(o)
        os.replace(tmp, out)
    return out


def build_hostsim(out_dir: str = None, force: bool = False, defines=(), flags=()) -> str:
    """The same kernel body compiled for the host CPU (libsfl_hostsim.so, OpenMP over envs): the
    parity tests' host build and bench.py's C++ CPU baseline -- never the product path.  Built
    in-tree so that it travels to the GPU box with the snapshot.  ``defines``: a tuning build (into
    another ``out_dir`` only; its build id differs, like build_hip's); ``flags`` likewise."""
    out_dir = out_dir or HERE
    defines, flags = list(defines), list(flags)
    if (defines or flags) and os.path.abspath(out_dir) == os.path.abspath(HERE):
        raise ValueError("build_hostsim: defines / flags are not built into the in-tree host build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.abspath(os.path.join(out_dir, "libsfl_hostsim.so"))
    if force or _stale(out, defines, flags):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fopenmp",
               f'-DSFL_BUILD_ID="{build_id(defines, flags)}"', f'-DSFL_BUILD_DEFS="{" ".join(sorted(defines))}"',
               f'-DSFL_BUILD_FLAGS="{" ".join(flags)}"'] + \
              [f"-D{d}" for d in defines] + list(flags) + ["-o", out + f".{os.getpid()}.tmp", os.path.join(CSRC, "sfl_hostsim.cpp")]
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(out + f".{os.getpid()}.tmp", out)
    return out


if __name__ == "__main__":
    print(build_hip(force="--force" in sys.argv, verbose=True))
