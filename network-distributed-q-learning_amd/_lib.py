"""ctypes binding of include/sfl.h.

The product loads ``libsfl.so`` (built for gfx950 by build.py) and nothing else:
there is no CPU fallback.  ``load(path)`` also serves the test-only host build
(``libsfl_hostsim.so``), which tests/ use to check the kernel body against the
oracle without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(HERE, "libsfl.so")
ABI_VERSION = 8  # include/sfl.h SFL_ABI_VERSION

P = C.POINTER


class MapDesc(C.Structure):
    _fields_ = [
        ("H", C.c_int32), ("W", C.c_int32), ("S", C.c_int32), ("T", C.c_int32), ("K", C.c_int32),
        ("max_episode_steps", C.c_int32), ("mf_rate", C.c_double), ("mf_min", C.c_int32), ("mf_max", C.c_int32),
        ("q_per_env", C.c_uint64), ("rows_per_env", C.c_uint32),
        ("grid", P(C.c_uint16)), ("cell_sw", P(C.c_int16)),
        ("sw_np", P(C.c_uint8)), ("sw_na", P(C.c_uint8)), ("act_src", P(C.c_uint8)), ("act_dst", P(C.c_uint8)),
        ("act_turn", P(C.c_uint8)), ("act_j", P(C.c_uint8)), ("first_other", P(C.c_uint8)),
        ("port_side", P(C.c_uint8)), ("slot_nroutes", P(C.c_uint8)), ("slot_route_act", P(C.c_uint8)),
        ("q_w", P(C.c_uint8)), ("port_nb", P(C.c_int16)), ("port_len", P(C.c_int16)), ("port_unique", P(C.c_int16)),
        ("q_off", P(C.c_uint64)), ("row_base", P(C.c_uint32)), ("dist", P(C.c_int32)),
        ("tr_ed", P(C.c_int32)), ("tr_la", P(C.c_int32)), ("tr_k", P(C.c_int32)), ("tr_target", P(C.c_int32)),
        ("tr_init_cell", P(C.c_int32)), ("tr_init_dist", P(C.c_int32)), ("tr_init_delay", P(C.c_int32)),
        ("tr_init_dir", P(C.c_uint8)), ("tr_init_port", P(C.c_int16)), ("delay_threshold", C.c_int32),
    ]


class HParams(C.Structure):
    _fields_ = [
        ("gamma", C.c_double), ("epsilon", C.c_double), ("epsilon_decay_rate", C.c_double), ("lr", C.c_double),
        ("lr_decay_rate", C.c_double), ("default_q", C.c_double), ("max_steps", C.c_int64), ("ntab", C.c_int32),
        ("eps_tab", P(C.c_double)), ("lr_tab", P(C.c_double)),
    ]


class RunArgs(C.Structure):
    _fields_ = [
        ("n_episodes", C.c_int32), ("exploit_freq", C.c_int32), ("stats_cap", C.c_int32), ("pad_", C.c_int32),
        ("cum_reward", P(C.c_double)), ("arrived", P(C.c_int32)), ("malfunctions", P(C.c_int32)),
        ("decisions", P(C.c_int32)), ("ticks", P(C.c_int32)), ("delays", P(C.c_int32)),
        ("exploit_cum", P(C.c_double)), ("exploit_arrived", P(C.c_int32)),
        ("trace", P(C.c_uint64)), ("trace_n", P(C.c_uint64)), ("trace_env", C.c_int32), ("trace_cap", C.c_int32),
    ]


class Counters(C.Structure):
    _fields_ = [("decisions", C.c_uint64), ("last_launch_decisions", C.c_uint64),
                ("last_launch_ticks", C.c_uint64), ("last_launch_alg_bytes", C.c_uint64),
                ("last_kernel_ms", C.c_double), ("kernel_variant", C.c_int32), ("group_lanes", C.c_int32)]


class EnvIO(C.Structure):
    """sfl_env_io (external-action mode)."""
    _fields_ = [("actions", P(C.c_int32)), ("agent", P(C.c_int32)), ("train", P(C.c_int32)), ("slot", P(C.c_int32)),
                ("state", P(C.c_uint32)), ("mask", P(C.c_uint32)), ("reward", P(C.c_int32)), ("now", P(C.c_int32)),
                ("next_switch", P(C.c_int32)), ("step_now", P(C.c_int32)), ("arrived", P(C.c_uint32)),
                ("malfunctions", P(C.c_int32)), ("delays", P(C.c_int32)), ("truncated", P(C.c_int32))]


EXPORTS = {
    "sfl_abi_version": (C.c_int, []),
    "sfl_build_id": (C.c_char_p, []),
    "sfl_last_error": (C.c_char_p, []),
    "sfl_device_count": (C.c_int, [P(C.c_int)]),
    "sfl_create": (C.c_int, [P(MapDesc), P(HParams), C.c_uint32, P(C.c_uint64), C.c_int, P(C.c_void_p)]),
    "sfl_destroy": (C.c_int, [C.c_void_p]),
    "sfl_learn_begin": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "sfl_apply_qinit": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32), P(C.c_double)]),
    "sfl_mark_exploit_done": (C.c_int, [C.c_void_p]),
    "sfl_learn": (C.c_int, [C.c_void_p, P(RunArgs)]),
    "sfl_test": (C.c_int, [C.c_void_p, P(RunArgs)]),
    "sfl_step": (C.c_int, [C.c_void_p, C.c_int64, P(C.c_uint64), P(C.c_double)]),
    "sfl_get_q": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_double), P(C.c_uint32)]),
    "sfl_set_q": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_double), P(C.c_uint32)]),
    "sfl_get_counters": (C.c_int, [C.c_void_p, P(Counters)]),
    "sfl_get_kernel_note": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    # external-action mode (aec.py) and the per-phase device time (distr_q.py timing accumulators)
    "sfl_env_begin": (C.c_int, [C.c_void_p]),
    "sfl_env_step": (C.c_int, [C.c_void_p, P(EnvIO)]),
    "sfl_get_phase_cycles": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_int32]),
    "sfl_get_env_state": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_int32), P(C.c_int32), P(C.c_uint64),
                                    P(C.c_int32), P(C.c_uint32)]),
    # Flatland-compatible malfunction stream (mfstream.py)
    "sfl_set_mf_schedule": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_uint8)]),
    "sfl_mf_schedule_flatland": (C.c_int, [P(C.c_uint32), C.c_int32, P(C.c_int32), C.c_int32, C.c_int32, C.c_double,
                                           C.c_int32, C.c_int32, C.c_int32, P(C.c_uint8)]),
    # graph-partitioned mode (partition.py)
    "sfl_part_config": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_int32), C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_uint32]),
    "sfl_part_record_sizes": (C.c_int, [P(C.c_uint32), P(C.c_uint32)]),
    "sfl_part_begin": (C.c_int, [C.c_void_p]),
    "sfl_part_local": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, P(C.c_uint64)]),
    "sfl_part_owner": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "sfl_part_counts": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_int32]),
    "sfl_part_set_caps": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sfl_get_sync_count": (C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint64)]),
    "sfl_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "sfl_part_set_local_rows": (C.c_int, [C.c_void_p, P(C.c_uint8)]),
    "sfl_part_get_q": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_double), P(C.c_uint32)]),
}


class SflError(RuntimeError):
    pass


class Lib:
    def __init__(self, path: str):
        if not os.path.exists(path):
            raise SflError(f"{path} not found — build it first (python -c 'import __graft_entry__ as g; g.build()')")
        self.path = path
        self.dll = C.CDLL(path)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args
        if self.dll.sfl_abi_version() != ABI_VERSION:
            raise SflError("ABI version mismatch")
        self.build_id = self.dll.sfl_build_id().decode()
        self.defines = ""
        self.flags = ""
        self.experimental = False

    def check_fresh(self, allow_experimental: bool = False):
        """Refuse a library that is not the product build of the sources in this tree: a stale build, or a
        tuning / experiment build (its -D defines or flags are part of its build id).  With
        ``allow_experimental`` a build of these sources with the defines it records is accepted
        (``self.defines`` then names them); experiment switches make its results invalid."""
        from . import build
        want = build.product_build_id()
        self.defines = build.built_defines(self.path) or ""
        self.flags = build.built_flags(self.path) or ""
        tuned = bool(self.defines or self.flags)
        if self.build_id == want and not tuned:
            self.experimental = False
            return
        if allow_experimental and tuned and self.build_id == build.build_id(self.defines.split(), self.flags.split()):
            self.experimental = True
            return
        what = f"defines: {self.defines or '-'}, flags: {self.flags or '-'}"
        if tuned and allow_experimental:
            raise SflError(f"{self.path} is stale: a tuning / experiment build ({what}) of other sources than the "
                           f"tree's (rebuild it)")
        if tuned:
            raise SflError(f"{self.path} is a tuning / experiment build ({what}), not the product library; set "
                           f"SFL_EXPERIMENTAL=1 (bench.py --experimental) to run it anyway")
        raise SflError(f"{self.path} is stale: built as {self.build_id[:12]}, the tree's product build is {want[:12]} "
                       f"(rebuild: python -c 'import __graft_entry__ as g; g.build()')")

    def check(self, rc: int, what: str):
        if rc != 0:
            raise SflError(f"{what}: {self.dll.sfl_last_error().decode(errors='replace')}")

    def device_count(self) -> int:
        n = C.c_int(0)
        self.dll.sfl_device_count(C.byref(n))
        return n.value


_product = None


def load_product() -> Lib:
    """The HIP library; raises if it is missing or no GPU is visible (no fallback)."""
    global _product
    if _product is None:
        # one HIP runtime per process: load torch's (it carries its own libamdhip64.so.7 / HSA runtime)
        # before libsfl.so resolves the same soname, so the library and torch's RCCL / allocator share it
        import torch  # noqa: F401

        # SFL_LIB: an alternative in-tree build of the same HIP sources (tuning sweeps); accepted only with
        # SFL_EXPERIMENTAL=1 unless it is the product build itself (check_fresh)
        lib = Lib(os.environ.get("SFL_LIB", PRODUCT_LIB))
        lib.check_fresh(allow_experimental=os.environ.get("SFL_EXPERIMENTAL") == "1")
        if lib.device_count() < 1:
            raise SflError("libsfl.so loaded but no HIP device is visible: the SwitchFL hot path runs on MI355X only")
        _product = lib
    return _product
