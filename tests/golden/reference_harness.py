"""TEST INFRASTRUCTURE (this container only): run the real reference ``switchfl`` code.

The reference imports flatland-rl, pettingzoo and gymnasium, none of which is
installed.  This harness registers minimal stand-in modules
under those names in ``sys.modules`` — all backed by ``oracle/flatland_lite.py``
(the frozen Flatland-semantics spec) and by numpy's own PCG64/SeedSequence for
gymnasium's ``Discrete`` — and then imports ``switchfl`` from
``/root/reference`` unchanged.  The reference's *patched* DistanceMap
(flatland_patch/distance_map.py) is imported from the reference too, so the
distance maps it produces pin the oracle's restatement.

Nothing here is used on the GPU box: the vectors it produces are committed
under tests/golden/ by make_golden.py.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from oracle import flatland_lite as fl  # noqa: E402


def _mod(name: str, **attrs) -> types.ModuleType:
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    parent, _, child = name.rpartition(".")
    if parent:
        setattr(sys.modules[parent], child, m)
    return m


class _Space:
    pass


class _Discrete(_Space):
    """gymnasium.spaces.Discrete: seed() builds Generator(PCG64(SeedSequence(seed)))."""

    def __init__(self, n, seed=None, start=0):
        self.n = int(n)
        self.start = int(start)
        self._np_random = None
        if seed is not None:
            self.seed(seed)

    def seed(self, seed=None):
        self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return [seed]

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    def sample(self, mask=None):
        if mask is not None:
            valid = mask == 1
            if np.any(valid):
                return self.start + self.np_random.choice(np.where(valid)[0])
            return self.start
        return self.start + self.np_random.integers(self.n)

    def contains(self, x):
        try:
            x = int(x)
        except Exception:
            return False
        return self.start <= x < self.start + self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class _MultiDiscrete(_Space):
    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec)
        self.dtype = dtype


class _AECEnv:
    """pettingzoo.AECEnv — only ``last`` and ``close`` are used by the reference."""

    def __init__(self, *a, **k):
        pass

    def last(self, observe=True):
        agent = self.agent_selection
        obs = self.observe(agent) if observe else None
        return (obs, self._cumulative_rewards[agent], self.terminations[agent],
                self.truncations[agent], self.infos[agent])

    def close(self):
        pass


class _MFP:
    def __init__(self, malfunction_rate=0.0, min_duration=0, max_duration=0):
        self.malfunction_rate, self.min_duration, self.max_duration = malfunction_rate, min_duration, max_duration


_installed = False


def install_stubs():
    global _installed
    if _installed:
        return
    _mod("flatland")
    _mod("flatland.core")
    _mod("flatland.core.grid")
    _mod("flatland.core.grid.grid4", Grid4TransitionsEnum=fl.Grid4TransitionsEnum)
    _mod("flatland.core.grid.grid4_utils", get_new_position=fl.get_new_position)
    _mod("flatland.envs")
    _mod("flatland.envs.step_utils")
    _mod("flatland.envs.step_utils.states", TrainState=fl.TrainState)
    _mod("flatland.envs.agent_utils", EnvAgent=fl.EnvAgent, Grid4TransitionsEnum=fl.Grid4TransitionsEnum)
    _mod("flatland.envs.rail_env", RailEnv=fl.RailEnv, RailEnvActions=fl.RailEnvActions)
    _mod("flatland.envs.rail_grid_transition_map", RailGridTransitionMap=fl.GridTransitionMap)
    _mod("flatland.envs.rail_trainrun_data_structures", Waypoint=fl.Waypoint)
    _mod("flatland.envs.rail_generators", sparse_rail_generator=None)
    _mod("flatland.envs.line_generators", sparse_line_generator=None)
    _mod("flatland.envs.malfunction_generators", MalfunctionParameters=_MFP, ParamMalfunctionGen=lambda p: p)
    _mod("flatland.utils")
    _mod("flatland.utils.rendertools", AgentRenderVariant=types.SimpleNamespace(AGENT_SHOWS_OPTIONS=0))
    _mod("pettingzoo", AECEnv=_AECEnv)
    _mod("gymnasium", Space=_Space)
    _mod("gymnasium.spaces", Discrete=_Discrete, MultiDiscrete=_MultiDiscrete, Space=_Space)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _installed = True


def patched_distance_map_cls():
    """The reference's patched DistanceMap (flatland_patch/distance_map.py), imported unchanged."""
    install_stubs()
    name = "flatland.envs.distance_map"
    if name in sys.modules and hasattr(sys.modules[name], "DistanceMap"):
        return sys.modules[name].DistanceMap
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, "flatland_patch", "distance_map.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m.DistanceMap


def make_rail_env(scenario):
    """flatland-lite RailEnv with the reference's patched DistanceMap installed."""
    install_stubs()
    DM = patched_distance_map_cls()
    env = fl.RailEnv(scenario)
    env.distance_map = DM(env.agents, env.height, env.width)
    env.reset()
    return env


def import_switchfl():
    install_stubs()
    patched_distance_map_cls()
    import logging
    logging.disable(logging.CRITICAL)
    switch_env = importlib.import_module("switchfl.switch_env")
    distr_q = importlib.import_module("switchfl.distr_q")
    return switch_env, distr_q
