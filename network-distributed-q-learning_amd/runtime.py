"""Batch runtime: E lock-step SwitchFL environments + learners on one GPU (one C-ABI handle).

Every env runs the same compiled map with its own seed — the seed the reference
passes both to ``env.reset(seed=...)`` (Flatland's malfunction stream) and to
``np.random.default_rng(seed)`` (the epsilon-greedy stream), distr_q.py:269, 296.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib, mfstream
from .compiler import CompiledMap, eps_table, lr_table, NTAB

P = C.POINTER


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(P(ctype))


def numpy_rng_state(seed: int) -> List[int]:
    """``np.random.default_rng(seed)`` bit-generator state as 5 uint64 words."""
    st = np.random.default_rng(int(seed)).bit_generator.state
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, (int(st["has_uint32"]) << 32) | int(st["uinteger"])]


class Batch:
    """Owns one device handle.  ``hp`` uses the reference's DistrQLearning argument names."""

    def __init__(self, cm: CompiledMap, hp: dict, seeds: Sequence[int], lib: Optional[_lib.Lib] = None,
                 device: int = 0, max_steps: int = 100_000, ntab: int = NTAB, malfunction_stream: str = "counter",
                 delay_threshold: int = 20):
        """``malfunction_stream``: "counter" (the counter-based draw of the frozen Flatland spec,
        oracle/flatland_lite.py) or "flatland" (ParamMalfunctionGen's np_random draw order, mfstream.py).
        ``delay_threshold``: StandardObserver's (observer.py:221)."""
        self.cm = cm
        self.malfunction_stream = mfstream.check_stream(malfunction_stream)
        self.hp = dict(hp)
        self.seeds = [int(s) for s in seeds]
        self.E = len(self.seeds)
        self.lib = lib or _lib.load_product()
        A = cm.arrays
        sc = cm.scenario
        self._keep = []  # arrays referenced by the descriptor until sfl_create copies them

        def arr(name, dtype):
            a = np.ascontiguousarray(A[name], dtype=dtype)
            self._keep.append(a)
            return a

        md = _lib.MapDesc()
        md.H, md.W, md.S, md.T, md.K = cm.H, cm.W, cm.S, cm.T, cm.K
        md.max_episode_steps = sc.max_episode_steps
        md.mf_rate, md.mf_min, md.mf_max = sc.malfunction_rate, sc.malfunction_min, sc.malfunction_max
        md.q_per_env, md.rows_per_env = cm.q_per_env, cm.rows_per_env
        md.delay_threshold = int(delay_threshold)
        spec = [("grid", np.uint16, C.c_uint16), ("cell_sw", np.int16, C.c_int16), ("sw_np", np.uint8, C.c_uint8),
                ("sw_na", np.uint8, C.c_uint8), ("act_src", np.uint8, C.c_uint8), ("act_dst", np.uint8, C.c_uint8),
                ("act_turn", np.uint8, C.c_uint8), ("act_j", np.uint8, C.c_uint8),
                ("first_other", np.uint8, C.c_uint8), ("port_side", np.uint8, C.c_uint8),
                ("slot_nroutes", np.uint8, C.c_uint8), ("slot_route_act", np.uint8, C.c_uint8),
                ("q_w", np.uint8, C.c_uint8), ("port_nb", np.int16, C.c_int16), ("port_len", np.int16, C.c_int16),
                ("port_unique", np.int16, C.c_int16), ("q_off", np.uint64, C.c_uint64),
                ("row_base", np.uint32, C.c_uint32), ("dist", np.int32, C.c_int32),
                ("tr_ed", np.int32, C.c_int32), ("tr_la", np.int32, C.c_int32), ("tr_k", np.int32, C.c_int32),
                ("tr_target", np.int32, C.c_int32), ("tr_init_cell", np.int32, C.c_int32),
                ("tr_init_dist", np.int32, C.c_int32), ("tr_init_delay", np.int32, C.c_int32),
                ("tr_init_dir", np.uint8, C.c_uint8), ("tr_init_port", np.int16, C.c_int16)]
        for name, dt, ct in spec:
            setattr(md, name, _ptr(arr(name, dt), ct))
        self.eps_tab = eps_table(hp["epsilon"], hp["epsilon_decay_rate"], ntab)
        self.lr_tab = lr_table(hp["lr"], hp["lr_decay_rate"], ntab)
        h = _lib.HParams()
        h.gamma, h.epsilon, h.epsilon_decay_rate = hp["gamma"], hp["epsilon"], hp["epsilon_decay_rate"]
        h.lr, h.lr_decay_rate, h.default_q = hp["lr"], hp["lr_decay_rate"], hp["default_q"]
        h.max_steps, h.ntab = int(max_steps), int(ntab)
        h.eps_tab, h.lr_tab = _ptr(self.eps_tab, C.c_double), _ptr(self.lr_tab, C.c_double)
        seeds_a = np.array(self.seeds, dtype=np.uint64)
        handle = C.c_void_p()
        self.lib.check(self.lib.dll.sfl_create(C.byref(md), C.byref(h), self.E, _ptr(seeds_a, C.c_uint64), device,
                                               C.byref(handle)), "sfl_create")
        self.h = handle
        self._keep = []
        note = C.create_string_buffer(256)
        self.lib.check(self.lib.dll.sfl_get_kernel_note(self.h, note, 256), "sfl_get_kernel_note")
        self.kernel_note = note.value.decode()
        if self.kernel_note:
            # the lane-per-env body is 15-45x slower than k_wave: say so, or refuse when asked to
            import os
            import warnings
            msg = f"this map runs the lane-per-env kernel (k_run), not k_wave: {self.kernel_note}"
            if os.environ.get("SFL_REQUIRE_WAVE") == "1":
                self.close()
                raise _lib.SflError(msg)
            warnings.warn(msg, RuntimeWarning, stacklevel=2)
        if self.malfunction_stream == "flatland":
            tab = mfstream.schedule(self.lib, sc, self.seeds)
            self.lib.check(self.lib.dll.sfl_set_mf_schedule(self.h, tab.shape[1], _ptr(tab, C.c_uint8)),
                           "sfl_set_mf_schedule")
        self.learn_calls = 0
        self.timed_kernel_ms = 0.0  # device time of the learn / test launches (the phase-timed ones)
        self.trace_env = None
        self.trace_cap = 1 << 16
        self.last_trace = None

    # ------------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.dll.sfl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _qinit_arrays(self):
        cm = self.cm
        keys = sorted(cm.qinit_rows)
        n = len(keys)
        port = np.array([4 * s + slot for s, slot, _ in keys], np.uint32)
        state = np.array([st for _, _, st in keys], np.uint32)
        vals = np.full((n, 4), np.nan)
        for i, k in enumerate(keys):
            row = cm.qinit_rows[k]
            vals[i, :len(row)] = row
        return n, port, state, vals

    def learn_begin(self):
        st = np.array([numpy_rng_state(s) for s in self.seeds], dtype=np.uint64)
        self.lib.check(self.lib.dll.sfl_learn_begin(self.h, _ptr(st, C.c_uint64)), "sfl_learn_begin")

    def apply_qinit(self):
        n, port, state, vals = self._qinit_arrays()
        self.lib.check(self.lib.dll.sfl_apply_qinit(self.h, n, _ptr(port, C.c_uint32), _ptr(state, C.c_uint32),
                                                    _ptr(vals, C.c_double)), "sfl_apply_qinit")

    def _run(self, fn, n_episodes, exploit_freq=0):
        """Run episodes; when ``self.trace_env`` is set, ``self.last_trace`` gets that env's decision trace."""
        E, T = self.E, self.cm.T
        cap = max(1, n_episodes)
        out = dict(cum_reward=np.zeros((cap, E)), arrived=np.zeros((cap, E), np.int32),
                   num_malfunctions=np.zeros((cap, E), np.int32), decisions=np.zeros((cap, E), np.int32),
                   ticks=np.zeros((cap, E), np.int32), delays=np.zeros((cap, T, E), np.int32),
                   cum_reward_exploit=np.zeros((cap, E)), arrived_trains_exploit=np.zeros((cap, E), np.int32))
        a = _lib.RunArgs()
        a.n_episodes, a.exploit_freq, a.stats_cap = n_episodes, exploit_freq, cap
        a.cum_reward = _ptr(out["cum_reward"], C.c_double)
        a.arrived = _ptr(out["arrived"], C.c_int32)
        a.malfunctions = _ptr(out["num_malfunctions"], C.c_int32)
        a.decisions = _ptr(out["decisions"], C.c_int32)
        a.ticks = _ptr(out["ticks"], C.c_int32)
        a.delays = _ptr(out["delays"], C.c_int32)
        a.exploit_cum = _ptr(out["cum_reward_exploit"], C.c_double)
        a.exploit_arrived = _ptr(out["arrived_trains_exploit"], C.c_int32)
        tr = tn = None
        if getattr(self, "trace_env", None) is not None:
            tr = np.zeros((self.trace_cap, 4), np.uint64)
            tn = np.zeros(1, np.uint64)
            a.trace, a.trace_n = _ptr(tr, C.c_uint64), _ptr(tn, C.c_uint64)
            a.trace_env, a.trace_cap = int(self.trace_env), int(self.trace_cap)
        self.lib.check(fn(self.h, C.byref(a)), fn.__name__)
        cnt = self.counters()
        if tr is None and cnt["kernel_variant"] > 0:
            # only the phase-timed instantiation stamps phase cycles: a traced launch (the TRACE kernel) or the
            # lane-per-env body adds kernel time without cycles, which would inflate phase_seconds
            self.timed_kernel_ms += cnt["last_kernel_ms"]
        if tr is not None:
            self.last_trace = tr[:min(int(tn[0]), self.trace_cap)]
        for k in list(out):
            out[k] = out[k][:n_episodes]
        return out

    def learn(self, n_episodes: int, exploit_freq: Optional[int] = None) -> Dict[str, np.ndarray]:
        """``DistrQLearning.learn`` for every env (distr_q.py:244-379); arrays are [episode][env]."""
        f = int(exploit_freq or 0)
        self.learn_begin()
        pre = None
        if f == 1 and n_episodes > 0:
            # the t=0 exploit round runs before __init_q_table (distr_q.py:278-300)
            pre = self.test(1)
            self.lib.check(self.lib.dll.sfl_mark_exploit_done(self.h), "sfl_mark_exploit_done")
        self.apply_qinit()
        out = self._run(self.lib.dll.sfl_learn, n_episodes, f)
        if pre is not None:
            out["cum_reward_exploit"][0] = pre["cum_reward"][0]
            out["arrived_trains_exploit"][0] = pre["arrived"][0]
        self.learn_calls += 1
        return out

    def test(self, n_episodes: int = 1) -> Dict[str, np.ndarray]:
        """``DistrQLearning.test`` greedy episodes (distr_q.py:184-241)."""
        return self._run(self.lib.dll.sfl_test, n_episodes)

    def step(self, decisions_per_env: int) -> Tuple[int, float]:
        """Advance every env by ``decisions_per_env`` learning decisions; returns (total decisions, kernel ms)."""
        n = C.c_uint64(0)
        ms = C.c_double(0.0)
        self.lib.check(self.lib.dll.sfl_step(self.h, int(decisions_per_env), C.byref(n), C.byref(ms)), "sfl_step")
        return int(n.value), float(ms.value)

    PHASES = ("tick", "observe", "egreedy", "apply", "post", "reset", "other")

    def phase_seconds(self) -> Dict[str, float]:
        """Device seconds per phase of the learn loop over this batch's learn / test launches so far: the
        launches' kernel time split by the sampled in-kernel phase cycles (sfl_get_phase_cycles; all zero on the
        lane-per-env body, which has no timers)."""
        cyc = np.zeros(8, np.uint64)
        self.lib.check(self.lib.dll.sfl_get_phase_cycles(self.h, _ptr(cyc, C.c_uint64), 8), "sfl_get_phase_cycles")
        total = float(cyc[7])
        sec = self.timed_kernel_ms * 1e-3
        return {k: (sec * float(cyc[i]) / total if total > 0 else 0.0) for i, k in enumerate(self.PHASES)}

    def counters(self) -> dict:
        c = _lib.Counters()
        self.lib.check(self.lib.dll.sfl_get_counters(self.h, C.byref(c)), "sfl_get_counters")
        return dict(decisions=c.decisions, last_launch_decisions=c.last_launch_decisions,
                    last_launch_ticks=c.last_launch_ticks, last_launch_alg_bytes=c.last_launch_alg_bytes,
                    last_kernel_ms=c.last_kernel_ms, kernel_variant=c.kernel_variant, group_lanes=c.group_lanes)

    # ---- Q-table export / import (the reference's pickle dict, distr_q.py:521-527) -------------
    def q_raw(self, env: int) -> Tuple[np.ndarray, np.ndarray]:
        q = np.zeros(self.cm.q_per_env)
        tw = (self.cm.rows_per_env + 31) // 32
        t = np.zeros(tw, np.uint32)
        self.lib.check(self.lib.dll.sfl_get_q(self.h, env, _ptr(q, C.c_double), _ptr(t, C.c_uint32)), "sfl_get_q")
        return q, t

    def set_q_raw(self, env: int, q: np.ndarray, touched: np.ndarray) -> None:
        """Overwrite one env's compact Q block and key-set bitmap (the layout of q_raw)."""
        q = np.ascontiguousarray(q, np.float64)
        touched = np.ascontiguousarray(touched, np.uint32)
        if q.size != self.cm.q_per_env or touched.size != (self.cm.rows_per_env + 31) // 32:
            raise ValueError("set_q_raw: arrays do not match the map's Q layout")
        self.lib.check(self.lib.dll.sfl_set_q(self.h, env, _ptr(q, C.c_double), _ptr(touched, C.c_uint32)),
                       "sfl_set_q")

    def q_dict(self, env: int) -> Dict[tuple, list]:
        """Touched rows as {observation tuple: [Q per action]} — the reference's ``q_table``."""
        cm = self.cm
        q, touched = self.q_raw(env)
        bits = np.unpackbits(touched.view(np.uint8), bitorder="little")[:cm.rows_per_env]
        rows = np.nonzero(bits)[0]
        A = cm.arrays
        dq = float(self.hp["default_q"])
        out = {}
        for s in range(cm.S):
            for slot in range(len(cm.ports[s])):
                g = 4 * s + slot
                base, nrows = int(A["row_base"][g]), (1 << len(cm.ports[s])) * cm.K * 3
                sel = rows[(rows >= base) & (rows < base + nrows)]
                if len(sel) == 0:
                    continue
                w = int(A["q_w"][g])
                off = int(A["q_off"][g])
                routes = [a for a, (src, _) in enumerate(cm.outcomes[s]) if src == slot] + [int(cm.n_actions[s]) - 1]
                for r in sel:
                    stt = int(r) - base
                    vals = q[off + stt * w: off + (stt + 1) * w]
                    full = [dq] * int(cm.n_actions[s])
                    for j, a in enumerate(routes):
                        full[a] = float(vals[j])
                    out[cm.obs_of_row(s, slot, stt)] = full
        return out

    def load_q_dict(self, env: int, table: Dict[tuple, list]):
        """Inverse of ``q_dict`` (``DistrQLearning.load``); rejects rows the compact layout cannot hold."""
        cm = self.cm
        A = cm.arrays
        dq = float(self.hp["default_q"])
        q = np.full(cm.q_per_env, dq)
        touched = np.zeros((cm.rows_per_env + 31) // 32, np.uint32)
        sidx = {sid: i for i, sid in enumerate(cm.switch_ids)}
        kidx = {st: i for i, st in enumerate(cm.stations)}
        for key, vals in table.items():
            s = sidx[(int(key[0]), int(key[1]))]
            P_ = len(cm.ports[s])
            sem = key[2:2 + P_]
            tgt = key[2 + P_:2 + 3 * P_]
            dl = key[2 + 3 * P_:2 + 4 * P_]
            slots = [i for i in range(P_) if dl[i] != -1]
            if len(slots) != 1:
                raise ValueError(f"row {key} has no unique in-port")
            slot = slots[0]
            k = kidx[(int(tgt[2 * slot]), int(tgt[2 * slot + 1]))]
            bits = sum(int(b) << j for j, b in enumerate(sem))
            stt = (bits * cm.K + k) * 3 + int(dl[slot])
            g = 4 * s + slot
            w, off = int(A["q_w"][g]), int(A["q_off"][g])
            routes = [a for a, (src, _) in enumerate(cm.outcomes[s]) if src == slot] + [int(cm.n_actions[s]) - 1]
            for a, v in enumerate(vals):
                if a not in routes and float(v) != dq:
                    raise ValueError(f"row {key}: action {a} does not leave from the in-port; not representable")
            for j, a in enumerate(routes):
                q[off + stt * w + j] = float(vals[a])
            rid = int(A["row_base"][g]) + stt
            touched[rid >> 5] |= np.uint32(1 << (rid & 31))
        self.lib.check(self.lib.dll.sfl_set_q(self.h, env, _ptr(q, C.c_double), _ptr(touched, C.c_uint32)),
                       "sfl_set_q")
