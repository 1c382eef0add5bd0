"""Post-run parity check of a sample of a batch's envs against the host build of the same kernel body.

A bench or multi-GPU run verifies itself: after the timed steps, every rank re-runs a spread sample of
its envs (same seeds, same step schedule) on ``libsfl_hostsim.so`` -- the kernel body compiled for the
host, itself pinned to the oracle and to the reference's golden traces by tests/ -- and compares the
Q-table, the key set (``__check_entry``, distr_q.py:47-57) and the env state (clock, phase, semaphore
table, train positions and bits) bit-exactly.  For the graph-partitioned mode the rank's owned rows of
the sampled envs are compared with a fused single-process run of those envs' seeds (the exchanged
successor lookup of distr_q.py:419-466 must leave every row as the fused loop would), and the env state
of the sampled envs it simulates.

The host build is a checker here, never the measured path: it runs after the timed region.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from .runtime import Batch


def spread(E: int, n: int = 8, stride: int = 1021) -> List[int]:
    """About n env indices spread over a batch of E (different blocks, CUs and XCDs), incl. the first and last."""
    if E <= n:
        return list(range(E))
    return sorted({(k * stride) % E for k in range(max(1, n - 2))} | {0, E - 1})


def env_state(b: Batch, env: int) -> Tuple[int, int, np.ndarray, np.ndarray, np.ndarray]:
    """(elapsed ticks, phase, semaphore records [4S] as 64-bit, train cells [T], train bits [T]) of one env."""
    cm = b.cm
    el, ph = C.c_int32(), C.c_int32()
    sem = np.zeros(4 * cm.S, np.uint64)
    pos = np.zeros(cm.T, np.int32)
    bits = np.zeros(cm.T, np.uint32)
    P = C.POINTER
    b.lib.check(b.lib.dll.sfl_get_env_state(b.h, env, C.byref(el), C.byref(ph), sem.ctypes.data_as(P(C.c_uint64)),
                                            pos.ctypes.data_as(P(C.c_int32)), bits.ctypes.data_as(P(C.c_uint32))),
                "sfl_get_env_state")
    return el.value, ph.value, sem, pos, bits


def _state_diff(a, b) -> List[str]:
    out = []
    for name, x, y in zip(("elapsed", "phase", "semaphores", "train cells", "train bits"), a, b):
        if not np.array_equal(np.asarray(x), np.asarray(y)):
            out.append(name)
    return out


def host_run(cm, hp: dict, seeds: Sequence[int], schedule: Sequence[int], host_lib: _lib.Lib, **kw) -> Batch:
    """The fused learn loop of ``seeds`` on the host build: learn_begin, the optimistic init, then one
    step per schedule entry (decisions per env), exactly as the device run was driven."""
    b = Batch(cm, hp, list(seeds), lib=host_lib, **kw)
    b.learn_begin()
    b.apply_qinit()
    for n in schedule:
        b.step(int(n))
    return b


def check_batch(b: Batch, hp: dict, pick: Sequence[int], schedule: Sequence[int], host_lib: _lib.Lib,
                **kw) -> List[str]:
    """Mismatches (empty: bit-equal) of envs ``pick`` of a device batch vs the host build's run of their seeds."""
    ref = host_run(b.cm, hp, [b.seeds[e] for e in pick], schedule, host_lib, **kw)
    bad = []
    try:
        for i, e in enumerate(pick):
            qg, tg = b.q_raw(e)
            qh, th = ref.q_raw(i)
            if not np.array_equal(qg, qh):
                bad.append(f"env {e}: Q-table ({int((qg != qh).sum())} cells)")
            if not np.array_equal(tg, th):
                bad.append(f"env {e}: key set")
            bad += [f"env {e}: {d}" for d in _state_diff(env_state(b, e), env_state(ref, i))]
    finally:
        ref.close()
    return bad


def check_partition(pb, hp: dict, pick_global: Sequence[int], seed_of, schedule: Sequence[int],
                    host_lib: _lib.Lib, **kw) -> List[str]:
    """Mismatches of a partitioned batch ``pb`` (partition.PartitionedBatch or CohortPipeline) for the job's global envs
    ``pick_global``: this rank's owned rows (and their key-set bits) vs a fused host run of those envs'
    seeds; the env state too for the sampled envs this rank simulates."""
    cm = pb.cm
    A = cm.arrays
    ref = host_run(cm, hp, [seed_of(g) for g in pick_global], schedule, host_lib, **kw)
    mk = pb.owned_mask()
    own_rows = np.zeros(cm.rows_per_env, bool)
    for s in range(cm.S):
        if pb.owner[s] != pb.rank:
            continue
        for slot in range(len(cm.ports[s])):
            g = 4 * s + slot
            base, n = int(A["row_base"][g]), (1 << len(cm.ports[s])) * cm.K * 3
            own_rows[base:base + n] = True
    bad = []
    try:
        for i, ge in enumerate(pick_global):
            q, t = pb.owned_q(ge)
            qr, tr = ref.q_raw(i)
            if not np.array_equal(q[mk], qr[mk]):
                bad.append(f"env {ge}: owned Q rows ({int((q[mk] != qr[mk]).sum())} cells)")
            bits = np.unpackbits(t.view(np.uint8), bitorder="little")[:cm.rows_per_env].astype(bool)
            rbits = np.unpackbits(tr.view(np.uint8), bitorder="little")[:cm.rows_per_env].astype(bool)
            if not np.array_equal(bits, rbits & own_rows):
                bad.append(f"env {ge}: owned key-set bits")
            sim = pb.sim_env(ge)  # (batch, local env) if this rank simulates it
            if sim is not None:
                bad += [f"env {ge}: {d}" for d in _state_diff(env_state(sim[0], sim[1]), env_state(ref, i))]
    finally:
        ref.close()
    return bad
