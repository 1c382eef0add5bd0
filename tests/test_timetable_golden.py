"""mapgen's timetable (earliest departure, latest arrival, max_episode_steps) against the reference's own
generator, flatland_patch/timetable_generators.py:23-136, run unchanged on the same trains and RandomState
by tests/golden/make_timetable_golden.py (vectors in tests/golden/timetable.json).  Covers the c1/c2/c3/c5
line grids, city maps and the reference's 80 x 80 sweep config (hyperparam_tuning.py:10-35, 5 seeds)."""
import json
import os

import pytest

from tests.golden import make_timetable_golden as mk

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "timetable.json")))


@pytest.mark.parametrize("case", GOLD, ids=[c["label"] for c in GOLD])
def test_timetable_matches_reference_generator(case):
    sc = mk.scenario(case["generator"], case["kwargs"])
    assert mk.n_cities_of(case["generator"], case["kwargs"], sc) == case["n_cities"]
    assert [t.earliest_departure for t in sc.trains] == case["earliest_departure"]
    assert [t.latest_arrival for t in sc.trains] == case["latest_arrival"]
    assert sc.max_episode_steps == case["max_episode_steps"]


def test_sweep_config_is_80_by_80():
    for case in GOLD:
        if case["label"].startswith("sweep80"):
            sc = mk.scenario(case["generator"], case["kwargs"])
            assert (sc.width, sc.height) == (80, 80) and len(sc.trains) == 15
