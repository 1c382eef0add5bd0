"""External-action mode: E SwitchFL environments stepped one decision per call by a policy on the host.

The reference's plugin surface between learner and env is the PettingZoo AEC protocol
(switchfl/switch_env.py:616-675): ``for agent in env.agent_iter(): obs, reward, term, trunc, info =
env.last(); ...; env.step(action)``, driven by any learner (distr_q.py:302-320).  The fused device loop
(runtime.Batch) runs the reference's own learner; this module exposes the env alone through
``sfl_env_begin`` / ``sfl_env_step`` (include/sfl.h): every call applies each env's action to the
observation the previous call emitted and runs the env on to its next decision (or episode end), on the
device, for all E envs at once.  ``ASyncSwitchEnv`` (env.py) wraps env 0 of an ``AECBatch`` in the
reference's single-env methods.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from .compiler import CompiledMap
from .runtime import Batch, _ptr

# the learner's hyper-parameters do not enter the env (no epsilon draw, no Q-table access)
ACTION_RESET = -2  # include/sfl.h SFL_ACTION_RESET: reset the env where it stands (env.reset() mid-episode)
_ENV_HP = dict(gamma=1.0, epsilon=0.0, epsilon_decay_rate=1.0, lr=0.0, lr_decay_rate=1.0, default_q=0.0)


class AECBatch:
    """E plain environments (no learner) on one device handle, stepped by ``step(actions)``.

    After each call, for env e: ``agent[e]`` is the deciding switch of its pending observation (-1: its
    episode ended in this call; the next call starts the next one), ``train``, ``slot``, ``state``
    (the observation index, ``observation(e)`` gives the reference's int64 vector), ``mask`` (action
    mask bits), ``reward`` (last()'s reward of (switch, train)), ``now``; for the action applied in this
    call ``next_switch`` and ``step_now`` (-1 if none); ``arrived`` (bitmask, 4 words); at an episode end
    ``malfunctions``, ``delays`` [T] and ``truncated``.
    """

    FIELDS = ("agent", "train", "slot", "state", "mask", "reward", "now", "next_switch", "step_now", "malfunctions",
              "truncated")

    def __init__(self, cm: CompiledMap, seeds: Sequence[int], lib: Optional[_lib.Lib] = None, device: int = 0,
                 max_steps: int = 100_000, malfunction_stream: str = "counter", delay_threshold: int = 20):
        self.cm = cm
        self.batch = Batch(cm, _ENV_HP, seeds, lib=lib, device=device, max_steps=max_steps, ntab=16,
                           malfunction_stream=malfunction_stream, delay_threshold=delay_threshold)
        self.lib = self.batch.lib
        self.E = self.batch.E
        E, T = self.E, cm.T
        self.out = {k: np.zeros(E, np.uint32 if k in ("state", "mask") else np.int32) for k in self.FIELDS}
        self.out["arrived"] = np.zeros((4, E), np.uint32)
        self.out["delays"] = np.zeros((T, E), np.int32)
        self._io = _lib.EnvIO()
        for k, ct in (("agent", C.c_int32), ("train", C.c_int32), ("slot", C.c_int32), ("state", C.c_uint32),
                      ("mask", C.c_uint32), ("reward", C.c_int32), ("now", C.c_int32), ("next_switch", C.c_int32),
                      ("step_now", C.c_int32), ("arrived", C.c_uint32), ("malfunctions", C.c_int32),
                      ("delays", C.c_int32), ("truncated", C.c_int32)):
            setattr(self._io, k, _ptr(self.out[k], ct))
        self._act = np.full(E, -1, np.int32)
        self.lib.check(self.lib.dll.sfl_env_begin(self.batch.h), "sfl_env_begin")

    def close(self):
        self.batch.close()

    def step(self, actions: Optional[Sequence[int]] = None) -> Dict[str, np.ndarray]:
        """Apply ``actions[e]`` to each env's pending observation (None / < 0: none; ``ACTION_RESET``: reset the env
        where it stands) and run every env to its next observation or episode end.  Returns the output arrays (views, valid until the next call)."""
        if actions is None:
            self._act[:] = -1
        else:
            a = np.asarray(actions, np.int64)
            if a.shape != (self.E,):
                raise ValueError(f"step: {a.shape} actions for {self.E} envs")
            # the reference asserts action_space(agent).contains(action) (switch_env.py:213-215)
            ag = self.out["agent"]
            pend = (ag >= 0) & (a >= 0)
            na = np.asarray(self.cm.n_actions, np.int64)[np.where(pend, ag, 0)]
            bad = np.nonzero(pend & (a >= na))[0]
            if len(bad):
                e = int(bad[0])
                raise ValueError(f"step: action {int(a[e])} of env {e} is outside switch {int(ag[e])}'s action space "
                                 f"Discrete({int(na[e])})")
            self._act[:] = np.where(a == ACTION_RESET, ACTION_RESET, np.where(a < 0, -1, a)).astype(np.int32)
        self._io.actions = _ptr(self._act, C.c_int32)
        self.lib.check(self.lib.dll.sfl_env_step(self.batch.h, C.byref(self._io)), "sfl_env_step")
        return self.out

    # ---- the reference's views of one env's pending decision ----------------------------------------
    def observation(self, e: int) -> np.ndarray:
        """observer.py:303-306: [r, c, sem[P], target[2P], delay[P]] (int64)."""
        s = int(self.out["agent"][e])
        if s < 0:
            return None
        return np.array(self.cm.obs_of_row(s, int(self.out["slot"][e]), int(self.out["state"][e])), np.int64)

    def action_mask(self, e: int) -> np.ndarray:
        s = int(self.out["agent"][e])
        n = int(self.cm.n_actions[s])
        m = int(self.out["mask"][e])
        return np.array([(m >> a) & 1 for a in range(n)], np.int8)

    def arrived_trains(self, e: int) -> List[int]:
        w = self.out["arrived"][:, e]
        return [h for h in range(self.cm.T) if (int(w[h >> 5]) >> (h & 31)) & 1]

    def agent_name(self, s: int) -> str:
        r, c = self.cm.switch_ids[s]
        return f"switch_{r}-{c}"

    def semaphores(self, e: int) -> dict:
        """Env e's semaphore table in the reference's format {port node: [owner, 'in'|'out', direction, t0, t1]}
        (rail_network.py:303-416; direction = map_direction(port), port_side)."""
        from .parity import env_state
        sem = env_state(self.batch, e)[2]
        side = self.cm.arrays["port_side"]
        out = {}
        for s, ports in enumerate(self.cm.ports):
            for j, node in enumerate(ports):
                r = int(sem[4 * s + j])
                if not (r >> 41) & 1:
                    continue
                t0 = (r & 0xFFFF) - ((r & 0x8000) << 1)
                t1 = ((r >> 16) & 0xFFFF) - (((r >> 16) & 0x8000) << 1)
                out[node] = [(r >> 32) & 0xFF, "in" if (r >> 40) & 1 else "out", int(side[4 * s + j]), t0, t1]
        return out

