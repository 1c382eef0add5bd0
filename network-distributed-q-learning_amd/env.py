"""``ASyncSwitchEnv``-shaped host object for a batch of lock-step SwitchFL environments.

The reference's ASyncSwitchEnv (switchfl/switch_env.py:605-678) is a PettingZoo AEC
env stepped one decision at a time from Python.  Here the whole agent_iter loop
runs on the GPU (csrc/sfl_core.h), so this class carries what the learner and the
scripts read from the env — the compiled switch network, agent names, action
spaces, ``max_steps``, the reset seed(s) and the timing accumulators
(test_model.py:76-82) — and owns the device batch.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

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

    def get_num_agents(self) -> int:
        return self.compiled.T

    def close(self):
        pass
