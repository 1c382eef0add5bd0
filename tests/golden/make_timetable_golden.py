"""TEST INFRASTRUCTURE (this container only): timetables from the reference's own generator.

Runs ``timetable_generator`` of flatland_patch/timetable_generators.py:23-136 -- imported unchanged
from /root/reference, with the reference's patched DistanceMap (flatland_patch/distance_map.py) and
minimal stand-ins for the Flatland modules it imports (reference_harness.py) -- on the trains of
mapgen scenarios, with the RandomState mapgen seeds its own timetable with, and records the earliest
departures, latest arrivals and max_episode_steps the reference computes.  tests/test_timetable_golden.py
checks mapgen's restatement (mapgen.timetable and the path lengths it is fed) against them.

Agents are given Flatland 4's line shape (waypoints = [[start], [target]]), so the generator takes its
intermediate-segment branch (timetable_generators.py:58-78), as it does for sparse_line_generator lines.
Usage: python tests/golden/make_timetable_golden.py   (writes tests/golden/timetable.json)
"""
from __future__ import annotations

import collections
import importlib
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from tests.golden import reference_harness as rh  # noqa: E402
from oracle import flatland_lite as fl  # noqa: E402

mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")

# (label, generator, kwargs): regenerated deterministically by the test
CASES = [
    ("c1", "make_config", dict(name="c1")),
    ("c2", "make_config", dict(name="c2")),
    ("c3", "make_config", dict(name="c3")),
    ("c5", "make_config", dict(name="c5")),
    ("c2_s3", "make_config", dict(name="c2", seed=3)),
    ("city4_s1", "generate_cities", dict(n_cities=4, n_trains=10, seed=1)),
    ("city6", "generate_cities", dict(n_cities=6, n_trains=12, seed=450565)),
    ("city9_s77", "generate_cities", dict(n_cities=9, n_trains=24, seed=77)),
] + [(f"sweep80_s{s}", "from_flatland_params", dict(width=80, height=80, max_num_cities=25, number_of_agents=15, seed=s))
     for s in (64, 65, 66, 67, 69)] + [  # hyperparam_tuning.py:10-35
    # round 4: the sweep's layout keys (max_rails_between_cities 2, max_rail_pairs_in_city 2) -> generate_city_grid
    (f"sweepgrid80_s{s}", "from_flatland_params", dict(width=80, height=80, max_num_cities=25, number_of_agents=15, seed=s,
                                                      max_rails_between_cities=2, max_rail_pairs_in_city=2))
    for s in (64, 65, 66, 67, 69)]


def scenario(gen, kw):
    kw = dict(kw)
    if gen == "make_config":
        return mapgen.make_config(kw.pop("name"), **kw)
    if gen == "generate_cities":
        return mapgen.generate_cities(**kw)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return mapgen.from_flatland_params(**kw)


def n_cities_of(gen, kw, sc):
    """The city count mapgen passes to its timetable (the reference reads len(city_positions))."""
    if gen == "make_config":
        return max(2, mapgen.CONFIGS[kw["name"]]["n_stations"])
    if gen == "generate_cities":
        return kw["n_cities"]
    return _cities_from_params(kw)


def _cities_from_params(kw):
    size = max(kw["width"], kw["height"])
    if kw.get("max_rails_between_cities") is not None:  # generate_city_grid: as many cities as fit, up to the cap
        pairs = kw.get("max_rail_pairs_in_city") or 1
        r_fit, c_fit = mapgen.city_grid_fit(size, 2 * pairs)
        cols = min(c_fit, kw["max_num_cities"])
        return min(r_fit, max(1, kw["max_num_cities"] // cols)) * cols
    n_fit = (size - 2 * mapgen.CITY_MARGIN - 1) // mapgen.CITY_SPACING + 1
    n_lines = 3
    while n_lines * (n_lines - 1) < kw["max_num_cities"] and n_lines < n_fit:
        n_lines += 1
    return min(kw["max_num_cities"], n_lines * (n_lines - 1))


class TTAgent:
    """The EnvAgent fields timetable_generator and DistanceMap.get_shortest_paths read."""

    def __init__(self, handle, initial_position, initial_direction, target, position=None, direction=None,
                 waypoints=None):
        self.handle = handle
        self.initial_position = tuple(initial_position)
        self.initial_direction = int(initial_direction)
        self.position = position
        self.direction = int(initial_direction if direction is None else direction)
        self.target = tuple(target)
        self.state = fl.TrainState.WAITING
        self.speed_counter = collections.namedtuple("SpeedCounter", "speed")(1.0)
        self.waypoints = waypoints or [[fl.Waypoint(self.initial_position, self.initial_direction)],
                                       [fl.Waypoint(self.target, None)]]
        self.earliest_departure = None
        self.latest_arrival = None


def reference_timetable_module():
    rh.install_stubs()
    DM = rh.patched_distance_map_cls()
    Timetable = collections.namedtuple("Timetable", "earliest_departures latest_arrivals max_episode_steps")
    rh._mod("flatland.envs.persistence")
    rh._mod("flatland.envs.timetable_utils", Timetable=Timetable)
    spec = importlib.util.spec_from_file_location("ref_timetable_generators",
                                                  os.path.join(rh.REF, "flatland_patch", "timetable_generators.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.EnvAgent = TTAgent  # the fake per-segment agents (timetable_generators.py:65-72)
    return mod, DM


def main():
    mod, DM = reference_timetable_module()
    out = []
    for label, gen, kw in CASES:
        sc = scenario(gen, kw)
        rail = fl.GridTransitionMap(sc.grid)
        agents = [TTAgent(h, t.initial_position, t.initial_direction, t.target) for h, t in enumerate(sc.trains)]
        dm = DM(agents, rail.height, rail.width)
        dm.reset(agents, rail)
        nc = n_cities_of(gen, kw, sc)
        rs = np.random.RandomState(sc.seed & 0x7FFFFFFF)
        tt = mod.timetable_generator(agents, dm, {"city_positions": [None] * nc}, rs)
        eds = [int(e[0]) for e in tt.earliest_departures]
        las = [int(l[-1]) for l in tt.latest_arrivals]
        out.append(dict(label=label, generator=gen, kwargs=kw, n_cities=nc, earliest_departure=eds, latest_arrival=las,
                        max_episode_steps=int(tt.max_episode_steps)))
        same = (eds == [t.earliest_departure for t in sc.trains] and las == [t.latest_arrival for t in sc.trains]
                and int(tt.max_episode_steps) == sc.max_episode_steps)
        print(f"{label}: {len(eds)} trains, max_episode_steps {tt.max_episode_steps}, mapgen {'==' if same else '!='} reference",
              flush=True)
    with open(os.path.join(HERE, "timetable.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
