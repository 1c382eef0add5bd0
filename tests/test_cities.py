"""Flatland-like city maps (mapgen.generate_cities): the generator's invariants,
and the host build of the kernel body against the oracle on a larger city map than the golden
fixtures (tests/golden/city*.json.gz, recorded from the reference itself, pin the smaller ones)."""
import importlib

import numpy as np
import pytest

from tests import hostsim
from oracle import sfl_oracle as so

mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")
comp = importlib.import_module("network-distributed-q-learning_amd.compiler")
runtime = importlib.import_module("network-distributed-q-learning_amd.runtime")
HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)


@pytest.mark.parametrize("n_cities,n_trains,seed", [(3, 4, 1), (6, 12, 450565), (9, 24, 77)])
def test_city_scenario_invariants(n_cities, n_trains, seed):
    sc = mapgen.generate_cities(n_cities, n_trains, seed=seed)
    again = mapgen.generate_cities(n_cities, n_trains, seed=seed)
    assert sc.to_json() == again.to_json()  # deterministic in the seed
    g = sc.grid_array()
    assert sc.height == sc.width and mapgen.strongly_connected(g)
    assert len(sc.trains) == n_trains
    starts = {t.initial_position for t in sc.trains}
    assert len(starts) == n_trains  # one train per start cell
    for t in sc.trains:
        assert t.target != t.initial_position
        assert 0 <= t.earliest_departure < t.latest_arrival <= sc.max_episode_steps
        # straight plain cells (a station or a start sits on a platform track)
        for cell in (t.initial_position, t.target):
            assert int(g[cell]) in (mapgen.pairs_to_bits({frozenset((mapgen.E, mapgen.W))}),)
    cm = comp.compile_scenario(sc)  # every junction is one of SwitchFL's switch classes
    assert cm.S >= 2 * n_cities and cm.T == n_trains


def test_city_map_host_build_matches_oracle():
    sc = mapgen.generate_cities(8, 20, seed=450565, malfunction=(0.01, 5, 15), name="city8")
    cm = comp.compile_scenario(sc)
    seeds = [450565, 3]
    b = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14)
    b.learn_begin()
    b.apply_qinit()
    total = 0
    for n in (50, 350):
        got, _ = b.step(n)
        assert got == n * len(seeds)
        total += n
    for e, seed in enumerate(seeds):
        env, model = so.build(sc, seed, HP, trace=False)
        so.run_decisions(model, total)
        assert b.q_dict(e) == model.q, f"env {e}"
    b.close()


def test_main_ini_uses_city_layout():
    sc = mapgen.from_flatland_params(60, 60, 4, 6, seed=450565)
    cm = comp.compile_scenario(sc)
    assert sc.width == sc.height and cm.T == 6
    assert len({t.target for t in sc.trains}) >= 2
    assert np.asarray(sc.grid).shape[0] >= 60


# ---- round 4: cities joined by rail paths of their own (mapgen.generate_city_grid) ----------------------
@pytest.mark.parametrize("rows,cols,rails,seed", [(2, 1, 1, 3), (3, 2, 2, 64), (7, 2, 2, 69)])
def test_city_grid_invariants(rows, cols, rails, seed):
    """Deterministic, strongly connected, one station per city on a platform, every switch a city's (throat, row
    chord, link end) or a link's diamond crossing: no junction joins two links; the sweep size fits 80 x 80."""
    sc = mapgen.generate_city_grid(rows, cols, 15, seed, rails=rails, size=80)
    assert sc.to_json() == mapgen.generate_city_grid(rows, cols, 15, seed, rails=rails, size=80).to_json()
    g = sc.grid_array()
    assert sc.height == sc.width == 80 and mapgen.strongly_connected(g)
    assert len({t.initial_position for t in sc.trains}) == 15
    straight = mapgen.pairs_to_bits({frozenset((mapgen.E, mapgen.W))})
    for t in sc.trains:
        assert int(g[t.initial_position]) == straight and int(g[t.target]) == straight
        assert 0 <= t.earliest_departure < t.latest_arrival <= sc.max_episode_steps
    cm = comp.compile_scenario(sc)
    assert cm.T == 15 and cm.K <= rows * cols
    # no four-way switching junction: every 4-port cell is a diamond crossing (N-S and E-W straight through)
    diamond = mapgen.pairs_to_bits({frozenset((mapgen.N, mapgen.S)), frozenset((mapgen.E, mapgen.W))})
    for r in range(g.shape[0]):
        for c in range(g.shape[1]):
            w = int(g[r, c])
            sides = {d for d in range(4) for h in range(4) if mapgen.transitions(w, h)[d]}
            if len(sides) == 4:
                assert w == diamond, (r, c)


def test_sweep_keys_take_the_city_grid():
    """hyperparam_tuning.py:17-25's [ENV] keys: as many cities as fit 80 x 80 (7 x 2 with up to 4 tracks), up to
    max_num_cities; layout="backbone" keeps round 3's layout (the citysweep_s5 fixture regenerates from it)."""
    from tests import _golden
    assert mapgen.city_grid_fit(80, 4) == (7, 2)
    sc = mapgen.from_flatland_params(80, 80, 25, 15, 64, max_rails_between_cities=2, max_rail_pairs_in_city=2)
    cm = comp.compile_scenario(sc)
    assert sc.width == 80 and cm.T == 15 and cm.K == 12
    few = mapgen.from_flatland_params(80, 80, 3, 15, 64, max_rails_between_cities=2, max_rail_pairs_in_city=2)
    assert comp.compile_scenario(few).K <= 3
    g = _golden.load("citysweep_s5")
    old = mapgen.from_flatland_params(60, 60, 6, 8, 5, malfunction=(0.02, 3, 8), max_rails_between_cities=2,
                                      max_rail_pairs_in_city=2, layout="backbone")
    assert old.to_json() == g["scenario_obj"].to_json()
    g = _golden.load("citygrid_s5")
    new = mapgen.from_flatland_params(60, 60, 6, 8, 5, malfunction=(0.02, 3, 8), max_rails_between_cities=2,
                                      max_rail_pairs_in_city=2)
    assert new.to_json() == g["scenario_obj"].to_json()


def test_city_grid_host_build_matches_oracle():
    sc = mapgen.generate_city_grid(3, 2, 12, 7, rails=2, size=80, malfunction=(0.01, 5, 15))
    cm = comp.compile_scenario(sc)
    seeds = [11, 450565]
    b = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14)
    b.learn_begin()
    b.apply_qinit()
    b.step(300)
    for e, seed in enumerate(seeds):
        env, model = so.build(sc, seed, HP, trace=False)
        so.run_decisions(model, 300)
        assert b.q_dict(e) == model.q, f"env {e}"
    b.close()
