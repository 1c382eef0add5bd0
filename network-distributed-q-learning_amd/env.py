"""``ASyncSwitchEnv``-shaped host object for a batch of lock-step SwitchFL environments.

The reference's ASyncSwitchEnv (switchfl/switch_env.py:605-678) is a PettingZoo AEC
env stepped one decision at a time from Python.  Here the whole agent_iter loop
runs on the GPU (csrc/sfl_core.h), so this class carries what the learner and the
scripts read from the env — the compiled switch network, agent names, action
spaces, ``max_steps``, the reset seed(s) and the timing accumulators
(test_model.py:76-82) — and owns the device batch.

It also speaks the AEC protocol itself for an external learner — ``reset(seed)``,
``agent_iter()``, ``last()``, ``step(action)``, ``observe(agent)`` (switch_env.py:93,
616-675) — on env 0 of an ``aec.AECBatch`` (the device's external-action mode: each
``step`` is one ``sfl_env_step`` launch).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np

from . import compiler, mapgen, mfstream
from . import observer as observer_mod


class Discrete:
    """Minimal stand-in for gymnasium.spaces.Discrete(n) (switch_agents.py:194-259)."""

    def __init__(self, n: int):
        self.n = int(n)

    def contains(self, x) -> bool:
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class ASyncSwitchEnv:
    """Batch of ``n_envs`` SwitchFL envs on one compiled map.

    ``rail_env`` may be a ``mapgen.Scenario``, a config name from ``mapgen.CONFIGS`` or a
    path to a scenario JSON file (Flatland's RailEnv is not available in this build).
    ``observer``: None or a ``StandardObserver`` (its ``delay_threshold`` reaches the kernels; see
    observer.py).  ``malfunction_stream="flatland"`` draws malfunctions in the order of Flatland's
    ``ParamMalfunctionGen`` on the reset-seeded ``np_random`` (mfstream.py) instead of the
    counter-based stream of the frozen spec.
    """

    def __init__(self, rail_env: Union[str, "mapgen.Scenario"], max_steps: int = 200, render_mode=None,
                 observer=None, seed: Optional[int] = None, n_envs: int = 1, device: int = 0,
                 malfunction_stream: str = "counter"):
        self.observer = observer
        self.delay_threshold = observer_mod.delay_threshold_of(observer)
        if isinstance(rail_env, str):
            sc = mapgen.make_config(rail_env) if rail_env in mapgen.CONFIGS else mapgen.Scenario.load(rail_env)
        else:
            sc = rail_env
        self.scenario = sc
        self.compiled = compiler.compile_scenario(sc)
        self.max_steps = int(max_steps)
        self.render_mode = render_mode
        self.seed = seed
        self.n_envs = int(n_envs)
        self.device = int(device)
        self.malfunction_stream = mfstream.check_stream(malfunction_stream)
        cm = self.compiled
        self.possible_agents: List[str] = [f"switch_{r}-{c}" for r, c in cm.switch_ids]
        self.agents = self.possible_agents
        self._spaces = {a: Discrete(int(n)) for a, n in zip(self.agents, cm.n_actions)}
        # timing accumulators read by the scripts (switch_env.py:67-73); filled from device timers
        self.flatland_step_time = 0.0
        self.step_time = 0.0
        self.last_time = 0.0
        self.action_selection_time = 0.0
        self.update_time = 0.0
        self.reset_time = 0.0
        self.reset_total_time = 0.0
        self.num_malfunctions = 0

    def action_space(self, agent: str) -> Discrete:
        return self._spaces[agent]

    # ---- the AEC protocol, env 0 of an external-action batch (switch_env.py:93, 616-675) ----------------
    def reset(self, seed: Optional[int] = None, options=None, lib=None):
        """Start an episode (switch_env.py:93-158) and run to its first decision.  A new seed (the
        malfunction stream's, like rail_env.reset(random_seed=seed)) starts a fresh device env; otherwise the
        env runs the same reset whether its episode ended or not (ACTION_RESET in the middle of one) and the
        trains' previous / source ports carry over, as in the reference."""
        from .aec import AECBatch, ACTION_RESET
        import time
        t0 = time.time()
        seed = int(seed if seed is not None else (self.seed if self.seed is not None else 0))
        aec = getattr(self, "_aec", None)
        if aec is None or seed != self._aec_seed or lib is not None:
            if aec is not None:
                aec.close()
            self._aec = AECBatch(self.compiled, [seed], lib=lib, device=self.device, max_steps=self.max_steps,
                                 malfunction_stream=self.malfunction_stream, delay_threshold=self.delay_threshold)
            self._aec_seed = seed
            out = self._aec.step(None)
        else:
            out = self._aec.out
            out = self._aec.step([ACTION_RESET] if out["agent"][0] >= 0 else None)
        self.terminated = self.truncated = False
        self._pending()
        self.reset_time += time.time() - t0
        self.reset_total_time += time.time() - t0
        return None

    def _pending(self):
        out = self._aec.out
        s = int(out["agent"][0])
        if s < 0:
            self.agent_selection = None
            self.active_train = None
            return
        self.agent_selection = self._aec.agent_name(s)
        self.active_train = int(out["train"][0])

    def agent_iter(self, max_iter: int = 2 ** 63):
        """Yield the deciding switch agent until the episode terminates or is truncated (switch_env.py:616-630)."""
        n = 0
        while not (self.terminated or self.truncated) and n < max_iter and self.agent_selection is not None:
            n += 1
            yield self.agent_selection

    def now(self) -> int:
        """rail_env._elapsed_steps at the pending observation."""
        return int(self._aec.out["now"][0])

    def observe(self, agent: str) -> np.ndarray:
        """observer.py:246-308 for the pending decision's agent."""
        if agent != self.agent_selection:
            raise ValueError(f"observe({agent}): only the deciding agent {self.agent_selection} has an observation")
        return self._aec.observation(0)

    def last(self, observe: bool = True):
        """AECEnv.last(): (observation, rewards by train, termination, truncation, info) of the deciding agent;
        the rewards map holds the active train's reward (switch_env.py:289: the reward its previous decision
        delivered at this switch)."""
        import time
        t0 = time.time()
        out = self._aec.out
        obs = self._aec.observation(0) if observe else None
        rew = {self.active_train: float(out["reward"][0])}
        info = {"action_mask": self._aec.action_mask(0), "active_train": self.active_train}
        self.last_time += time.time() - t0
        return obs, rew, bool(self.terminated), bool(self.truncated), info

    def step(self, action) -> dict:
        """switch_env.py:632-666: apply the action, move the trains if no switch is active, and return
        {"next_switch": (r, c), "arrived_trains": [handles]}."""
        import time
        if self.terminated or self.truncated or action is None or self.agent_selection is None:
            return {}
        if not self.action_space(self.agent_selection).contains(action):  # switch_env.py:213-215
            raise AssertionError(f"action {action} outside {self.action_space(self.agent_selection)}")
        t0 = time.time()
        out = self._aec.step([int(action)])
        nxt = int(out["next_switch"][0])
        self.step_elapsed = int(out["step_now"][0])
        arrived = self._aec.arrived_trains(0)
        if out["agent"][0] < 0:  # the episode ended in this step
            self.truncated = bool(out["truncated"][0])
            self.terminated = not self.truncated
            self.num_malfunctions = int(out["malfunctions"][0])
            self.train_to_last_node_delays = [int(x) for x in out["delays"][:, 0]]
        self._pending()
        self.step_time += time.time() - t0
        self.flatland_step_time += self._aec.batch.counters()["last_kernel_ms"] * 1e-3
        return {"next_switch": tuple(self.compiled.switch_ids[nxt]), "arrived_trains": arrived}

    def semaphores(self) -> dict:
        """The port reservation table of env 0 in the reference's format (rail_network.semaphores)."""
        return self._aec.semaphores(0)

    def get_num_agents(self) -> int:
        return self.compiled.T

    def close(self):
        aec = getattr(self, "_aec", None)
        if aec is not None:
            aec.close()
            self._aec = None
