"""``DistrQLearning``-shaped learner over the device batch (switchfl/distr_q.py:11-527).

Same constructor arguments, ``learn`` / ``test`` / ``save`` / ``load`` / ``q_table``, and
the same output files (distr_q.py:237-239, 287-294, 368-375):

    cum_reward.npz, arrived_trains.npz, delays.npz, trains_at_dest.npz,
    num_malfunctions.npz, [cum_reward_exploit.npz, arrived_trains_exploit.npz],
    checkpoint_<t>.pkl + *_checkpoint_<t>.npz every ``checkpoint_freq`` episodes

With ``env.n_envs == 1`` the files have exactly the reference's shapes; with a batch
of E envs (the MI355X use case: a seed sweep in lock-step) every array gets a leading
env axis and env e runs with seed ``seed + e``.
"""
from __future__ import annotations

import os
import pickle
import time
from typing import Dict, List, Optional

import numpy as np

from . import runtime
from .env import ASyncSwitchEnv


class DistrQLearning:
    def __init__(self, env: ASyncSwitchEnv, gamma=1.0, epsilon=0.4, epsilon_decay_rate=0.0, lr=0.4,
                 lr_decay_rate=0.0, default_q=0.0, seed=450565, lib=None):
        self.env = env
        self.gamma = gamma
        self.initial_epsilon = epsilon
        self.epsilon_decay_rate = epsilon_decay_rate
        self.initial_lr = lr
        self.lr_decay_rate = lr_decay_rate
        self.default_q = default_q
        self.seed = seed
        self.optimal_init = 500.0
        self.destination_bonus = 1000.0
        self.hp = dict(gamma=gamma, epsilon=epsilon, epsilon_decay_rate=epsilon_decay_rate, lr=lr,
                       lr_decay_rate=lr_decay_rate, default_q=default_q)
        seeds = [int(seed) + e for e in range(env.n_envs)]
        self.batch = runtime.Batch(env.compiled, self.hp, seeds, lib=lib, device=env.device, max_steps=env.max_steps,
                                   malfunction_stream=getattr(env, "malfunction_stream", "counter"),
                                   delay_threshold=getattr(env, "delay_threshold", 20))

    # ------------------------------------------------------------------
    @property
    def q_table(self) -> Dict[tuple, list]:
        """Env 0's Q-table as the reference's dict {observation tuple: [Q per action]}."""
        return self.batch.q_dict(0)

    def q_tables(self) -> List[Dict[tuple, list]]:
        return [self.batch.q_dict(e) for e in range(self.batch.E)]

    def _squeeze(self, a):
        return a[0] if self.batch.E == 1 else a

    def _save(self, out_dir, name, arr):
        np.savez_compressed(os.path.join(out_dir, name), x=arr)

    def _timing(self, t0):
        """The reference's accumulators (switch_env.py:67-73, distr_q.py:271-273, 304-358), from the device's
        phase timers: flatland_step_time = the Flatland ticks, last_time = observe, action_selection_time =
        epsilon-greedy, update_time = the post step (Q update, pending map, destination bonus), reset_time =
        reset_total_time = the episode resets, step_time = apply + ticks (env.step incl. _move_trains_to_switch).
        Without timers (the lane-per-env body) step_time is the call's wall time and flatland_step_time its
        kernel time."""
        ph = self.batch.phase_seconds()
        prev = getattr(self, "_phase_prev", None) or {k: 0.0 for k in ph}
        d = {k: ph[k] - prev[k] for k in ph}
        self._phase_prev = ph
        if sum(d.values()) > 0:
            self.env.flatland_step_time += d["tick"]
            self.env.last_time += d["observe"]
            self.env.action_selection_time += d["egreedy"]
            self.env.update_time += d["post"]
            self.env.reset_time += d["reset"]
            self.env.reset_total_time += d["reset"]
            self.env.step_time += d["apply"] + d["tick"]
        else:
            c = self.batch.counters()
            self.env.step_time += time.time() - t0
            self.env.flatland_step_time += c["last_kernel_ms"] * 1e-3

    # ------------------------------------------------------------------
    def learn(self, num_episodes: int, out_dir: str, checkpoint_freq: int, exploit_freq: Optional[int] = None):
        """distr_q.py:244-379 for every env of the batch."""
        t0 = time.time()
        b = self.batch
        E, T = b.E, b.cm.T
        f = int(exploit_freq or 0)
        b.learn_begin()
        pre = None
        if f == 1 and num_episodes > 0:
            pre = b.test(1)
            b.lib.check(b.lib.dll.sfl_mark_exploit_done(b.h), "sfl_mark_exploit_done")
        # checkpoints are written at the start of episode t with (t+1) % checkpoint_freq == 0, after
        # that episode's exploit round (distr_q.py:278-294): when both fall on t, the greedy round
        # runs here (its max_action key-set inserts belong in the checkpoint) and the kernel skips it.
        # __init_q_table runs after episode 0's reset (distr_q.py:296-300), i.e. after checkpoint_1.
        stops = [t for t in range(num_episodes) if checkpoint_freq and (t + 1) % checkpoint_freq == 0]
        qinit_pending = True
        if not stops or stops[0] != 0:
            b.apply_qinit()
            qinit_pending = False
        cum = np.zeros((num_episodes, E))
        arrived = np.zeros((num_episodes, E), np.int32)
        delays = np.zeros((num_episodes, T, E))
        mfs = np.zeros((num_episodes, E), np.int32)
        cum_x = np.zeros((num_episodes, E))
        arr_x = np.zeros((num_episodes, E), np.int32)
        pre_x = {}
        done = 0
        for stop in stops + [num_episodes]:
            n = stop - done
            if n > 0:
                out = b._run(b.lib.dll.sfl_learn, n, f)
                cum[done:stop] = out["cum_reward"]
                arrived[done:stop] = out["arrived"]
                delays[done:stop] = out["delays"]
                mfs[done:stop] = out["num_malfunctions"]
                cum_x[done:stop] = out["cum_reward_exploit"]
                arr_x[done:stop] = out["arrived_trains_exploit"]
                done = stop
            if stop < num_episodes:
                t = stop
                if f and (t + 1) % f == 0 and not (t == 0 and pre is not None):
                    x = b.test(1)
                    b.lib.check(b.lib.dll.sfl_mark_exploit_done(b.h), "sfl_mark_exploit_done")
                    pre_x[t] = (x["cum_reward"][0], x["arrived"][0])
                self.save(os.path.join(out_dir, f"checkpoint_{t + 1}.pkl"))
                self._save(out_dir, f"cum_reward_checkpoint_{t + 1}.npz", self._env_major(cum))
                self._save(out_dir, f"arrived_trains_checkpoint_{t + 1}.npz", self._env_major(arrived[:t]))
                self._save(out_dir, f"delays_checkpoint_{t + 1}.npz", self._env_major(delays[:t], delays=True))
                # the reference resets trains_at_destination just before saving it (distr_q.py:285 vs 293)
                self._save(out_dir, f"trains_at_dest_checkpoint_{t + 1}.npz", np.array([]))
                self._save(out_dir, f"num_malfunctions_checkpoint_{t + 1}.npz", self._env_major(mfs[:t]))
                if qinit_pending:
                    b.apply_qinit()
                    qinit_pending = False
        if pre is not None:
            cum_x[0] = pre["cum_reward"][0]
            arr_x[0] = pre["arrived"][0]
        for t, (c_, a_) in pre_x.items():  # (the kernel's rows for these episodes were not written)
            cum_x[t] = c_
            arr_x[t] = a_
        self._save(out_dir, "cum_reward.npz", self._env_major(cum))
        self._save(out_dir, "arrived_trains.npz", self._env_major(arrived))
        self._save(out_dir, "delays.npz", self._env_major(delays, delays=True))
        self._save(out_dir, "trains_at_dest.npz", self._trains_at_dest())
        self._save(out_dir, "num_malfunctions.npz", self._env_major(mfs))
        if f:
            sel = (np.arange(num_episodes) + 1) % f == 0
            self._save(out_dir, "cum_reward_exploit.npz", self._env_major(cum_x[sel]))
            self._save(out_dir, "arrived_trains_exploit.npz", self._env_major(arr_x[sel]))
        self.env.num_malfunctions = self._squeeze(mfs[-1]) if num_episodes else 0
        self._timing(t0)
        return dict(cum_reward=cum, arrived_trains=arrived, delays=delays, num_malfunctions=mfs,
                    cum_reward_exploit=cum_x, arrived_trains_exploit=arr_x)

    def _env_major(self, a, delays=False):
        """[episode, (train,) env] -> reference shape (E == 1) or env-leading axis."""
        a = np.asarray(a)
        if delays:
            a = a.astype(np.float64)
            a = np.moveaxis(a, -1, 0)  # [E, episode, train]
        else:
            a = np.moveaxis(a, -1, 0)  # [E, episode]
        return a[0] if self.batch.E == 1 else a

    def _trains_at_dest(self):
        res = []
        for e in range(self.batch.E):
            _, _, _, _, tr_bits = self._env_state(e)
            res.append([h for h, bits in enumerate(tr_bits) if ((bits >> 2) & 7) == 6])
        return np.array(res[0]) if self.batch.E == 1 else np.array(res, dtype=object)

    def _env_state(self, e):
        import ctypes as C
        cm = self.batch.cm
        el = np.zeros(1, np.int32)
        ph = np.zeros(1, np.int32)
        sem = np.zeros(4 * cm.S, np.uint64)
        pos = np.zeros(cm.T, np.int32)
        bits = np.zeros(cm.T, np.uint32)
        P = C.POINTER
        self.batch.lib.check(self.batch.lib.dll.sfl_get_env_state(
            self.batch.h, e, el.ctypes.data_as(P(C.c_int32)), ph.ctypes.data_as(P(C.c_int32)),
            sem.ctypes.data_as(P(C.c_uint64)), pos.ctypes.data_as(P(C.c_int32)),
            bits.ctypes.data_as(P(C.c_uint32))), "sfl_get_env_state")
        return int(el[0]), int(ph[0]), sem, pos, bits

    def test(self, out_dir, plot=False, save_outputs=True):
        """distr_q.py:184-241: one greedy episode per env; returns (cum_reward, arrived, delays)."""
        t0 = time.time()
        out = self.batch.test(1)
        cum = self._squeeze(out["cum_reward"][0])
        arrived = self._squeeze(out["arrived"][0])
        delays = out["delays"][0].T.astype(np.float64)  # [E, T]
        delays = delays[0].tolist() if self.batch.E == 1 else delays
        if save_outputs:
            print(f"Terminated in {self._squeeze(out['decisions'][0])} steps "
                  f"({self._squeeze(out['ticks'][0])} flatland steps), cumulative reward = {cum}")
            print(f"Arrived trains: {arrived} / {self.batch.cm.T}")
            print(f"Delays: {delays}")
            print(f"Num malfunctions: {self._squeeze(out['num_malfunctions'][0])}")
            self._save(out_dir, "cum_reward.npz", cum)
            self._save(out_dir, "trains_at_dest.npz", self._trains_at_dest())
            self._save(out_dir, "delays.npz", delays)
        self._timing(t0)
        return cum, arrived, delays

    def save(self, filename: str, mode: str = "pickle"):
        """distr_q.py:492-508 — pickle of the Q dict (a list of dicts for a batch)."""
        if mode != "pickle":
            raise NotImplementedError("only mode='pickle' is supported (the reference defines no csv/parquet dumper)")
        obj = self.q_table if self.batch.E == 1 else self.q_tables()
        with open(filename, "wb") as f:
            pickle.dump(obj, f)

    def load(self, filename: str):
        """distr_q.py:510-527 — a file written by ``save`` (our own pickle)."""
        with open(filename, "rb") as f:
            obj = pickle.load(f)
        tables = obj if isinstance(obj, list) else [obj] * self.batch.E
        for e, t in enumerate(tables[: self.batch.E]):
            self.batch.load_q_dict(e, t)
