"""The CPU oracle (oracle/sfl_oracle.py) against vectors recorded from the real reference."""
import numpy as np
import pytest

from tests import _golden
from oracle import sfl_oracle as so

CASES = _golden.cases()


def _q_dict(items):
    return {tuple(k): v for k, v in items}


def _run(name):
    g = _golden.load(name)
    hp = g["hparams"]
    env, model = so.build(g["scenario_obj"], g["seed"], hp, max_steps=hp.get("max_steps", 100_000))
    return g, env, model


@pytest.mark.parametrize("name", CASES)
def test_tables(name):
    g, env, model = _run(name)
    net = env.net
    assert [s["id"] for s in g["tables"]] == [list(s) for s in net.switch_ids]
    for s in g["tables"]:
        sw = net.switches[tuple(s["id"])]
        assert [list(p) for p in sw.ports] == s["ports"], s["id"]
        assert [[list(a), list(b)] for a, b in sw.outcomes] == s["outcomes"]
        assert [[int(x) for x in p] for p in sw.plans] == s["plans"]
        assert sw.n_actions == s["n_actions"]
        for p, (nsw, npt), L, prev in zip(sw.ports, s["neighbor"], s["seg_len"], s["prev_node"]):
            assert list(net.neighbor[p][0]) == nsw and list(net.neighbor[p][1]) == npt
            assert net.seg_len[p] == L
            assert list(net.prev_node[p]) == prev


@pytest.mark.parametrize("name", CASES)
def test_distance_init_ports_qinit(name):
    g, env, model = _run(name)
    d = np.where(np.isinf(env.dist), -1, env.dist).astype(np.int64)
    assert np.array_equal(d, np.array(g["distance"]))
    env.reset(seed=g["seed"])
    assert [[list(env.next_port[h]), env.next_port_dist[h]] for h in range(len(env.rail_env.agents))] == \
        [[p, n] for p, n in g["init_ports"]]
    model.init_q_table()
    assert model.q == _q_dict(g["q_init"])


@pytest.mark.parametrize("name", CASES)
def test_learn_and_test_trace(name):
    g, env, model = _run(name)
    out = model.learn(g["n_episodes"], exploit_freq=g["exploit_freq"])
    ev, gev = model.events, g["learn"]["events"]
    for i, (a, b) in enumerate(zip(ev, gev)):
        assert a == b, f"event {i}: oracle {a} != reference {b}"
    assert len(ev) == len(gev)
    for k, v in g["learn"]["outputs"].items():
        assert out[k] == v, k
    assert model.q == _q_dict(g["learn"]["q_final"])
    model.events = []
    cr, arr, delays = model.test()
    assert model.events == g["test"]["events"]
    assert (cr, arr, [float(x) for x in delays]) == (g["test"]["cum_reward"], g["test"]["arrived"], g["test"]["delays"])
    assert model.q == _q_dict(g["test"]["q_final"])
