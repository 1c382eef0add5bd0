"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Flatland-semantics restatement ("flatland-lite"): the part of the hot path
that the reference delegates to the third-party ``flatland-rl`` package
(``RailEnv.step`` / ``reset``, ``rail.check_action_on_agent``,
``rail.get_valid_move_actions_``, ``EnvAgent``, ``TrainState``).  flatland-rl
is not installed in this container and is unpinned in the reference
(requirements.txt:5), so these semantics are **parity unpinned** against real
Flatland: this file is the frozen spec that both the HIP kernels and the CPU
oracle implement (DESIGN.md §"Flatland semantics").  It follows the
Flatland-3/4 design the reference's call sites imply:

* speed-1 trains, state machine WAITING → READY_TO_DEPART → MOVING/STOPPED,
  MALFUNCTION(_OFF_MAP), DONE; removal at target, ``arrival_time`` set
  (call sites switch_env.py:343-348, 659-660);
* ``check_action_on_agent(action, (pos, dir))`` returns
  ``(new_cell_valid, (new_pos, new_dir), transition_valid, action)``
  (switch_env.py:319-329, 443-454; reward_func.py:45-53);
* ``get_valid_move_actions_(dir, pos)`` yields RailEnvNextAction in
  [left, forward, right] order (switch_env.py:538; distance_map.py:210);
* conflicts: the lowest handle wins a contested cell; a train may enter an
  occupied cell only if its occupant leaves it in the same step (chains
  resolve, swaps and cycles block);
* malfunctions: counter-based draw ``mf_draw(seed, tick, handle)`` (so every
  episode reset with the same seed replays the same malfunctions, like
  Flatland's ``reset(random_seed=seed)``), rate/min/max as
  ``MalfunctionParameters`` (test_model.py:14-19).

The module also backs the stub ``flatland.*`` modules used by
tests/golden/make_golden.py to run the real reference code in this
container.
"""
from __future__ import annotations

from collections import namedtuple
from enum import IntEnum
from typing import Dict, List, Optional, Tuple

import numpy as np

M64 = (1 << 64) - 1


class RailEnvActions(IntEnum):
    DO_NOTHING = 0
    MOVE_LEFT = 1
    MOVE_FORWARD = 2
    MOVE_RIGHT = 3
    STOP_MOVING = 4

    def is_moving_action(self) -> bool:
        return self in (RailEnvActions.MOVE_LEFT, RailEnvActions.MOVE_FORWARD, RailEnvActions.MOVE_RIGHT)


class Grid4TransitionsEnum(IntEnum):
    NORTH = 0
    EAST = 1
    SOUTH = 2
    WEST = 3


class TrainState(IntEnum):
    WAITING = 0
    READY_TO_DEPART = 1
    MALFUNCTION_OFF_MAP = 2
    MOVING = 3
    STOPPED = 4
    MALFUNCTION = 5
    DONE = 6

    def is_off_map_state(self) -> bool:
        return self in (TrainState.WAITING, TrainState.READY_TO_DEPART, TrainState.MALFUNCTION_OFF_MAP)

    def is_on_map_state(self) -> bool:
        return self in (TrainState.MOVING, TrainState.STOPPED, TrainState.MALFUNCTION)

    def is_malfunction_state(self) -> bool:
        return self in (TrainState.MALFUNCTION, TrainState.MALFUNCTION_OFF_MAP)


Waypoint = namedtuple("Waypoint", ["position", "direction"])
RailEnvNextAction = namedtuple("RailEnvNextAction", ["action", "next_position", "next_direction"])

DELTA = ((-1, 0), (0, 1), (1, 0), (0, -1))


def get_new_position(position, movement):
    return (position[0] + DELTA[movement][0], position[1] + DELTA[movement][1])


# ---------------------------------------------------------------------------
# counter-based malfunction draws (identical arithmetic in csrc/sfl_device.h)
# ---------------------------------------------------------------------------

def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def mf_draw(seed: int, tick: int, handle: int) -> int:
    return mix64((seed & M64) * 0x9E3779B97F4A7C15 + (tick & M64) * 0xD1B54A32D192ED03
                 + (handle & M64) * 0x8CB92BA72F3D8DD7 + 0x632BE59BD9B4E019)


def gym_seed_key(seed: int):
    """``flatland.utils.seeding.np_random(seed)``'s argument to ``RandomState.seed`` (gym's seeding:
    create_seed -> hash_seed (sha512 of str(seed), first 8 bytes) -> _int_list_from_bigint)."""
    import hashlib
    import struct
    a = int(seed) % (1 << 64)
    b = hashlib.sha512(str(a).encode("utf8")).digest()[:8] + b"\0" * 4
    big = 0
    for i, v in enumerate(struct.unpack("<3I", b)):
        big += v << (32 * i)
    ints = []
    while big > 0:
        big, mod = divmod(big, 1 << 32)
        ints.append(mod)
    return ints or [0]


def mf_uniform(z: int) -> float:
    return (z >> 11) * (1.0 / 9007199254740992.0)


def mf_duration(z: int, lo: int, hi: int) -> int:
    return lo + mix64(z ^ 0xA0761D6478BD642F) % (hi - lo + 1)


# ---------------------------------------------------------------------------
# rail grid
# ---------------------------------------------------------------------------

class GridTransitionMap:
    """16-bit Flatland cell transitions on an H x W grid."""

    def __init__(self, grid):
        self.grid = np.asarray(grid, dtype=np.int64)
        self.height, self.width = self.grid.shape

    def get_full_transitions(self, row, column):
        return int(self.grid[row, column])

    def get_transitions(self, *args):
        """``get_transitions(((r, c), dir))`` or ``get_transitions((r, c), dir)`` or ``(r, c, dir)``."""
        if len(args) == 1:
            (r, c), d = args[0]
        elif len(args) == 2:
            (r, c), d = args
        else:
            r, c, d = args
        nib = (int(self.grid[r, c]) >> ((3 - int(d)) * 4)) & 0xF
        return ((nib >> 3) & 1, (nib >> 2) & 1, (nib >> 1) & 1, nib & 1)

    def get_transition(self, cell_dir, direction):
        (r, c), d = cell_dir
        return (int(self.grid[r, c]) >> ((3 - int(d)) * 4 + (3 - int(direction)))) & 1

    def check_bounds(self, pos):
        return 0 <= pos[0] < self.height and 0 <= pos[1] < self.width

    def is_dead_end(self, pos):
        w = int(self.grid[pos[0], pos[1]])
        # a dead end: exactly one connected side (never produced by the scenario generator)
        sides = set()
        for d in range(4):
            for e, ok in enumerate(self.get_transitions(pos, d)):
                if ok:
                    sides.add(e)
        return w != 0 and len(sides) == 1

    def check_action_on_agent(self, action, position_direction):
        position, direction = position_direction
        direction = int(direction)
        trans = self.get_transitions(position, direction)
        n = sum(trans)
        new_dir = direction
        valid = None
        if action == RailEnvActions.MOVE_LEFT:
            new_dir = direction - 1
            if n <= 1:
                valid = False
        elif action == RailEnvActions.MOVE_RIGHT:
            new_dir = direction + 1
            if n <= 1:
                valid = False
        new_dir %= 4
        if action == RailEnvActions.MOVE_FORWARD and n == 1:
            new_dir = trans.index(1)
            valid = True
        new_pos = get_new_position(position, new_dir)
        new_cell_valid = self.check_bounds(new_pos) and self.get_full_transitions(*new_pos) > 0
        if valid is None:
            valid = bool(trans[new_dir])
        return new_cell_valid, (new_pos, new_dir), bool(valid), action

    def get_valid_move_actions_(self, agent_direction, agent_position):
        d = int(agent_direction)
        trans = self.get_transitions(agent_position, d)
        n = sum(trans)
        out = []
        for i in (-1, 0, 1):
            nd = (d + i) % 4
            if not trans[nd]:
                continue
            if n == 1:
                act = RailEnvActions.MOVE_FORWARD
            elif i == 0:
                act = RailEnvActions.MOVE_FORWARD
            elif i == 1:
                act = RailEnvActions.MOVE_RIGHT
            else:
                act = RailEnvActions.MOVE_LEFT
            out.append(RailEnvNextAction(act, get_new_position(agent_position, nd), nd))
        return out


def action_valid(rail: GridTransitionMap, action, pos, direction) -> bool:
    ncv, _, tv, _ = rail.check_action_on_agent(action, (pos, direction))
    return bool(ncv and tv)


# ---------------------------------------------------------------------------
# agents + env
# ---------------------------------------------------------------------------

class MalfunctionHandler:
    def __init__(self):
        self.malfunction_down_counter = 0

    @property
    def in_malfunction(self):
        return self.malfunction_down_counter > 0


class EnvAgent:
    def __init__(self, initial_position, initial_direction, target, earliest_departure, latest_arrival, handle):
        self.initial_position = tuple(int(x) for x in initial_position)
        self.initial_direction = int(initial_direction)
        self.direction = int(initial_direction)
        self.target = tuple(int(x) for x in target)
        self.earliest_departure = int(earliest_departure)
        self.latest_arrival = int(latest_arrival)
        self.handle = handle
        self.position = None
        self.old_position = None
        self.old_direction = None
        self.arrival_time = None
        self.moving = False
        self.state = TrainState.WAITING
        self.saved_action = None
        self.malfunction_handler = MalfunctionHandler()

    def reset(self):
        self.position = None
        self.direction = self.initial_direction
        self.old_position = None
        self.old_direction = None
        self.arrival_time = None
        self.moving = False
        self.state = TrainState.WAITING
        self.saved_action = None
        self.malfunction_handler.malfunction_down_counter = 0


def _next_state(state: TrainState, s: dict) -> TrainState:
    """Flatland TrainStateMachine transitions (one step)."""
    if state == TrainState.WAITING:
        if s["in_malfunction"]:
            return TrainState.MALFUNCTION_OFF_MAP
        return TrainState.READY_TO_DEPART if s["ed_reached"] else TrainState.WAITING
    if state == TrainState.READY_TO_DEPART:
        if s["in_malfunction"]:
            return TrainState.MALFUNCTION_OFF_MAP
        return TrainState.MOVING if s["valid_move"] else TrainState.READY_TO_DEPART
    if state == TrainState.MALFUNCTION_OFF_MAP:
        if s["counter_complete"]:
            return TrainState.READY_TO_DEPART if s["ed_reached"] else TrainState.WAITING
        return TrainState.MALFUNCTION_OFF_MAP
    if state == TrainState.MOVING:
        if s["in_malfunction"]:
            return TrainState.MALFUNCTION
        if s["stop_given"]:
            return TrainState.STOPPED
        if s["target_reached"]:
            return TrainState.DONE
        if s["conflict"]:
            return TrainState.STOPPED
        return TrainState.MOVING
    if state == TrainState.STOPPED:
        if s["in_malfunction"]:
            return TrainState.MALFUNCTION
        return TrainState.MOVING if s["valid_move"] else TrainState.STOPPED
    if state == TrainState.MALFUNCTION:
        if s["counter_complete"]:
            return TrainState.MOVING if s["valid_move"] else TrainState.STOPPED
        return TrainState.MALFUNCTION
    return TrainState.DONE


def motion_check(positions: List[Optional[Tuple[int, int]]], desired: List[Optional[Tuple[int, int]]],
                 movers: List[bool]) -> List[bool]:
    """Least fixed point of 'i may move'.  ``movers[i]``: i wants to change cell (or enter the map)."""
    T = len(positions)
    occ = {}
    for i in range(T):
        if positions[i] is not None:
            occ[positions[i]] = i
    winner = {}
    for i in range(T):
        if movers[i]:
            c = desired[i]
            if c not in winner:
                winner[c] = i  # handle order: lowest handle first
    allowed = [False] * T
    changed = True
    while changed:
        changed = False
        for i in range(T):
            if not movers[i] or allowed[i] or winner[desired[i]] != i:
                continue
            j = occ.get(desired[i])
            if j is None or (movers[j] and allowed[j]):
                allowed[i] = True
                changed = True
    return allowed


class RailEnv:
    """Speed-1 Flatland-semantics environment over a ``mapgen.Scenario``."""

    def __init__(self, scenario, remove_agents_at_target: bool = True, mf_stream: str = "counter"):
        """``mf_stream``: "counter" (``mf_draw``) or "flatland": ParamMalfunctionGen's draws on the
        env's ``np_random`` (numpy's RandomState, reseeded at every reset by a nonzero seed), for every
        agent at every step in handle order -- ``rand() < 1 - exp(-rate)`` then ``randint(lo, hi + 1) + 1``
        -- after the timetable's ``randint(0, departure_window_max)`` per agent at reset
        (timetable_generators.py:113-115).  Parity with real Flatland unpinned (Flatland absent)."""
        assert mf_stream in ("counter", "flatland")
        self.mf_stream = mf_stream
        self.np_random = None
        self.scenario = scenario
        self.rail = GridTransitionMap(scenario.grid)
        self.height, self.width = self.rail.height, self.rail.width
        self._max_episode_steps = int(scenario.max_episode_steps)
        self.malfunction_rate = float(scenario.malfunction_rate)
        self.malfunction_min = int(scenario.malfunction_min)
        self.malfunction_max = int(scenario.malfunction_max)
        self.agents: List[EnvAgent] = [
            EnvAgent(t.initial_position, t.initial_direction, t.target, t.earliest_departure, t.latest_arrival, h)
            for h, t in enumerate(scenario.trains)]
        self._elapsed_steps = 0
        self.random_seed = 0
        self.dones = {}
        self.distance_map = None  # installed by the user (oracle restatement or the reference's patched DistanceMap)

    def get_num_agents(self):
        return len(self.agents)

    def reset(self, regenerate_rail=True, regenerate_schedule=True, random_seed=None, **kw):
        self.random_seed = 0 if random_seed is None else int(random_seed)
        self._elapsed_steps = 0
        if self.mf_stream == "flatland" and random_seed:
            self.np_random = np.random.RandomState()
            self.np_random.seed(gym_seed_key(self.random_seed))
            mes = self._max_episode_steps
            lam = mes - int(mes * 0.05)
            for t in self.scenario.trains:  # the timetable generator's draws
                self.np_random.randint(0, max(lam - (t.latest_arrival - t.earliest_departure), 1))
        # the same map + line every reset (the reference reseeds with a fixed seed: distr_q.py:195, 296)
        self.agents.sort(key=lambda a: a.handle)
        for h, a in enumerate(self.agents):
            a.reset()
        self.dones = {h: False for h in range(len(self.agents))}
        self.dones["__all__"] = False
        if self.distance_map is not None and hasattr(self.distance_map, "reset"):
            self.distance_map.reset(self.agents, self.rail)
        return None, {}

    def render(self, *a, **k):
        return None

    def _preprocess(self, action, a: EnvAgent):
        try:
            action = RailEnvActions(int(action))
        except ValueError:
            action = RailEnvActions.DO_NOTHING
        if action == RailEnvActions.DO_NOTHING and a.state == TrainState.MOVING:
            action = RailEnvActions.MOVE_FORWARD
        if a.state == TrainState.WAITING:
            action = RailEnvActions.DO_NOTHING
        pos, d = (a.position, a.direction) if a.position is not None else (a.initial_position, a.initial_direction)
        if action in (RailEnvActions.MOVE_LEFT, RailEnvActions.MOVE_RIGHT) and not action_valid(self.rail, action, pos, d):
            action = RailEnvActions.MOVE_FORWARD
        if action.is_moving_action() and not action_valid(self.rail, action, pos, d):
            action = RailEnvActions.STOP_MOVING
        return action

    def step(self, action_dict: Dict[int, int]):
        self._elapsed_steps += 1
        t = self._elapsed_steps
        T = len(self.agents)
        desired = [None] * T
        desired_dir = [None] * T
        movers = [False] * T
        pa = [None] * T
        for a in self.agents:
            h = a.handle
            a.old_position, a.old_direction = a.position, a.direction
            mh = a.malfunction_handler
            if self.mf_stream == "flatland":
                if self.np_random is None:
                    raise ValueError("the flatland malfunction stream needs reset(random_seed=<nonzero>)")
                p = 1.0 - float(np.exp(-self.malfunction_rate)) if self.malfunction_rate > 0 else 0.0
                n = 0
                if self.np_random.rand() < p:
                    n = int(self.np_random.randint(self.malfunction_min, self.malfunction_max + 1)) + 1
                if a.state != TrainState.DONE and mh.malfunction_down_counter == 0 and n > 0:
                    mh.malfunction_down_counter = n
            elif a.state != TrainState.DONE and mh.malfunction_down_counter == 0 and self.malfunction_rate > 0.0:
                z = mf_draw(self.random_seed, t, h)
                if mf_uniform(z) < self.malfunction_rate:
                    mh.malfunction_down_counter = mf_duration(z, self.malfunction_min, self.malfunction_max) + 1
            act = self._preprocess(action_dict.get(h, RailEnvActions.DO_NOTHING), a)
            if act.is_moving_action() and a.saved_action is None and a.state != TrainState.DONE:
                a.saved_action = act
            update_allowed = (mh.malfunction_down_counter == 0) and act != RailEnvActions.STOP_MOVING
            if a.state == TrainState.DONE:
                want, wdir = a.position, a.direction
            elif a.position is None and a.saved_action is not None:
                want, wdir = a.initial_position, a.initial_direction
                movers[h] = True
            elif a.saved_action is not None and update_allowed:
                _, (want, wdir), _, _ = self.rail.check_action_on_agent(a.saved_action, (a.position, a.direction))
                act = a.saved_action
                movers[h] = want != a.position
            else:
                want, wdir = a.position, a.direction
            desired[h], desired_dir[h], pa[h] = want, wdir, act
        allowed = motion_check([a.position for a in self.agents], desired, movers)
        all_done = True
        for a in self.agents:
            h = a.handle
            mh = a.malfunction_handler
            ma = False if mh.in_malfunction else (allowed[h] if movers[h] else False)
            sig = dict(in_malfunction=mh.in_malfunction,
                       counter_complete=mh.malfunction_down_counter == 0,
                       ed_reached=t >= a.earliest_departure,
                       stop_given=pa[h] == RailEnvActions.STOP_MOVING,
                       valid_move=pa[h].is_moving_action() and ma,
                       target_reached=a.position == a.target,
                       conflict=not ma)
            prev = a.state
            a.state = _next_state(a.state, sig)
            ma = ma and a.state != TrainState.DONE
            if a.state.is_on_map_state():
                if prev.is_off_map_state():
                    a.position, a.direction = a.initial_position, a.initial_direction
                elif ma:
                    a.position, a.direction = desired[h], desired_dir[h]
                    if a.position == a.target:
                        a.state = TrainState.DONE
            if a.state == TrainState.DONE and a.arrival_time is None:
                a.arrival_time = t
                a.position = None
            if mh.malfunction_down_counter > 0:
                mh.malfunction_down_counter -= 1
            if a.position is not None:
                a.saved_action = None
            a.moving = a.state == TrainState.MOVING
            self.dones[h] = a.state == TrainState.DONE
            all_done &= a.state == TrainState.DONE
        if all_done or t >= self._max_episode_steps:
            for h in range(T):
                self.dones[h] = True
            self.dones["__all__"] = True
        info = {"malfunction": {a.handle: a.malfunction_handler.malfunction_down_counter for a in self.agents},
                "state": {a.handle: a.state for a in self.agents}}
        return {}, {a.handle: 0.0 for a in self.agents}, dict(self.dones), info
